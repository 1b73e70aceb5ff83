"""FactoryVecEnv: the SB3 VecEnv surface over N arenas resident on one MI355X.

Replaces ``make_vec_env(lambda: Monitor(Env(**env_kwargs)), n_envs, vec_env_cls=SubprocVecEnv)``
(/root/reference/src/learning.py:98-100): same ``num_envs / observation_space / action_space /
reset() / step_async() / step_wait() / step() / get_attr / set_attr / env_method / close / seed``
surface and the same auto-reset + ``infos[i]["terminal_observation"]`` + Monitor
``infos[i]["episode"] = {"r", "l", "t"}`` semantics, but every arena lives in HBM and one HIP launch
advances all of them (no worker processes, no pickled pipes).  Observations / rewards / dones are
torch ROCm tensors; ``return_numpy=True`` gives numpy like SB3.
"""
import ctypes as C
import time

import numpy as np

from . import _lib

# the env classes of src/environments.py (class hierarchy at environments.py:10-22)
ENV_CLASSES = {
    "FactoryManipulationEnv": _lib.FM_ENV_FACTORY,
    "AllFullRLProgressRewardEnv": _lib.FM_ENV_ALLFULLRL_PROGRESS,
    "SingleFullRLProgressRewardEnv": _lib.FM_ENV_SINGLEFULLRL_PROGRESS,
    "SingleDeltaProgressRewardEnv": _lib.FM_ENV_SINGLEDELTA_PROGRESS,
    "AllDeltaProgressRewardEnv": _lib.FM_ENV_ALLDELTA_PROGRESS,
    "PauseIKToggleEnv": _lib.FM_ENV_PAUSE_IK_TOGGLE,
    "BackupIKToggleEnv": _lib.FM_ENV_BACKUP_IK_TOGGLE,
}
TOGGLE_CLASSES = ("PauseIKToggleEnv", "BackupIKToggleEnv")

# BaseEnv.__init__ defaults (base_env.py:15-35); ProgressRewardEnv weights of the saved runs
# (runs/rk5rxnav.json env_kwargs)
DEFAULT_KWARGS = dict(
    num_arms=2, max_num_objects=10, seed=42, initial_conveyor_speed=0.1, conveyor_acceleration=0.001,
    pt_time=0.2, force_contact_threshold=200.0, control_frequency=10, spawn_freq=1 / 10,
    spawn_freq_increase=1.001, gripper_to_closest_cube_reward_factor=0.2,
    closest_cube_to_bucket_reward_factor=0.4, small_action_norm_reward_factor=0.0, base_reward=0.4,
)
_IGNORED_KWARGS = {"render_mode", "width", "height", "camera_id", "camera_name", "default_camera_config",
                   "max_geom", "visual_options"}


class Box:
    """minimal gymnasium.spaces.Box stand-in (gymnasium is not a dependency)"""

    def __init__(self, low, high, shape, dtype):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

    def sample(self, rng=np.random):
        lo = np.broadcast_to(self.low, self.shape)
        hi = np.broadcast_to(self.high, self.shape)
        return rng.uniform(lo, hi).astype(self.dtype)

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"


class MultiDiscrete:
    """minimal gymnasium.spaces.MultiDiscrete stand-in (IKTogglingEnv.action_space, environments.py:551)"""

    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.dtype(np.int64)

    def sample(self, rng=np.random):
        return rng.integers(0, self.nvec) if hasattr(rng, "integers") else rng.randint(0, self.nvec)

    def __repr__(self):
        return f"MultiDiscrete({self.nvec})"


class FactoryVecEnv:
    def __init__(self, num_envs, env_class="AllFullRLProgressRewardEnv", env_kwargs=None, device=0,
                 precision="fp32", seeds=None, return_numpy=False, max_contacts=0, solver_tolerance=0.0,
                 solver_iterations=0):
        import torch

        self.torch = torch
        kw = dict(DEFAULT_KWARGS)
        kw.update({k: v for k, v in (env_kwargs or {}).items() if k not in _IGNORED_KWARGS})
        if env_class not in ENV_CLASSES:
            raise ValueError(f"env_class {env_class!r} not implemented on the GPU path; "
                             f"available: {sorted(ENV_CLASSES)}")
        self.env_class = env_class
        self.env_kwargs = kw
        L = _lib.load()
        cfg = _lib.FmConfig()
        L.fm_config_default(C.byref(cfg))
        cfg.num_arenas = int(num_envs)
        cfg.num_arms = int(kw["num_arms"])
        cfg.max_num_objects = int(kw["max_num_objects"])
        cfg.env_class = ENV_CLASSES[env_class]
        cfg.precision = _lib.FM_FP64 if precision == "fp64" else _lib.FM_FP32
        cfg.max_contacts = int(max_contacts)
        if solver_tolerance > 0:  # 0 = the precision's default (fm_create)
            cfg.solver_tolerance = float(solver_tolerance)
        if solver_iterations > 0:
            cfg.solver_iterations = int(solver_iterations)
        for k in ["initial_conveyor_speed", "conveyor_acceleration", "pt_time", "force_contact_threshold",
                  "control_frequency", "spawn_freq", "spawn_freq_increase", "gripper_to_closest_cube_reward_factor",
                  "closest_cube_to_bucket_reward_factor", "small_action_norm_reward_factor", "base_reward"]:
            setattr(cfg, k, float(kw[k]))
        if seeds is None:
            seeds = [int(kw["seed"])] * int(num_envs)
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        if len(seeds) != num_envs:
            raise ValueError("need one seed per arena")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        h = C.c_void_p()
        _lib.check(L.fm_create(C.byref(cfg), self.device.index or 0,
                               seeds.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(h)))
        self._h = h
        self._L = L
        self.num_envs = int(num_envs)
        self.precision = precision
        self.obs_dim = L.fm_obs_dim(h)
        self.act_dim = L.fm_act_dim(h)
        self.observation_space = Box(-np.inf, np.inf, (self.obs_dim,), np.float32)
        if env_class in TOGGLE_CLASSES:
            self.action_space = MultiDiscrete([2] * self.act_dim)
        else:
            self.action_space = Box(-1.0, 1.0, (self.act_dim,), np.float32)
        self.return_numpy = return_numpy
        dev = self.device
        n = self.num_envs
        self.obs = torch.zeros(n, self.obs_dim, dtype=torch.float32, device=dev)
        self.rewards = torch.zeros(n, dtype=torch.float32, device=dev)
        self.terminated = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.scores = torch.zeros(n, 2, dtype=torch.int32, device=dev)
        self.num_obj = torch.zeros(n, dtype=torch.int32, device=dev)
        self.play_time = torch.zeros(n, dtype=torch.float64, device=dev)
        self.conveyor_speed = torch.zeros(n, dtype=torch.float64, device=dev)
        self.out_of_reach = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.force_terminate = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.terminal_obs = torch.zeros(n, self.obs_dim, dtype=torch.float32, device=dev)
        self.ep_return = torch.zeros(n, dtype=torch.float64, device=dev)
        self.ep_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self.terminal_scores = torch.zeros(n, 2, dtype=torch.int32, device=dev)
        self._info = _lib.FmInfo(*[t.data_ptr() for t in (
            self.scores, self.num_obj, self.play_time, self.conveyor_speed, self.out_of_reach, self.force_terminate,
            self.terminal_obs, self.ep_return, self.ep_len, self.terminal_scores)])
        self._actions = None
        self._stream_bound = -1
        self.ep_score_history = [[] for _ in range(n)]
        self._t0 = [time.time()] * n

    # ------------------------------------------------------------------ core API
    def _bind_stream(self):
        """run on torch's current stream so action / observation tensors are ordered with torch work"""
        s = self.torch.cuda.current_stream(self.device)
        if self._stream_bound != s.cuda_stream:
            _lib.check(self._L.fm_set_stream(self._h, C.c_void_p(s.cuda_stream) if s.cuda_stream else None))
            self._stream_bound = s.cuda_stream

    def reset(self, mask=None):
        self._bind_stream()
        mptr = None
        if mask is not None:
            m = self.torch.as_tensor(mask, dtype=self.torch.uint8, device=self.device).contiguous()
            mptr = C.c_void_p(m.data_ptr())
        _lib.check(self._L.fm_reset(self._h, mptr, C.c_void_p(self.obs.data_ptr())))
        now = time.time()
        self._t0 = [now] * self.num_envs
        return self.obs.cpu().numpy() if self.return_numpy else self.obs

    def step_tensors(self, actions):
        """device fast path: actions float32 [N, act_dim] tensor -> (obs, reward, terminated, truncated) tensors"""
        a = actions
        if not (self.torch.is_tensor(a) and a.device == self.device and a.dtype == self.torch.float32
                and a.is_contiguous()):
            # MultiDiscrete int actions (toggle classes) become 0.0 / 1.0
            a = self.torch.as_tensor(np.asarray(a) if not self.torch.is_tensor(a) else a, device=self.device)
            a = a.to(self.torch.float32).contiguous()
        if a.numel() == 0:  # FactoryManipulationEnv: no action entries; the ABI still takes a pointer
            a = self.torch.zeros(max(self.num_envs, 1), dtype=self.torch.float32, device=self.device)
        self._actions = a
        self._bind_stream()
        _lib.check(self._L.fm_step(self._h, C.c_void_p(a.data_ptr()), C.c_void_p(self.obs.data_ptr()),
                                   C.c_void_p(self.rewards.data_ptr()), C.c_void_p(self.terminated.data_ptr()),
                                   C.c_void_p(self.truncated.data_ptr()), C.byref(self._info)))
        return self.obs, self.rewards, self.terminated, self.truncated

    def step_async(self, actions):
        self._pending = actions

    def step_wait(self):
        obs, rew, term, trunc = self.step_tensors(self._pending)
        dones = term.bool() | trunc.bool()
        infos = self._infos(dones)
        if self.return_numpy:
            return obs.cpu().numpy(), rew.cpu().numpy(), dones.cpu().numpy(), infos
        return obs, rew, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _infos(self, dones):
        d = dones.cpu().numpy()
        sc = self.scores.cpu().numpy()
        pt = self.play_time.cpu().numpy()
        cs = self.conveyor_speed.cpu().numpy()
        oor = self.out_of_reach.cpu().numpy()
        ft = self.force_terminate.cpu().numpy()
        infos = []
        idx = np.nonzero(d)[0]
        term = {}
        if len(idx):
            tobs = self.terminal_obs[idx].cpu().numpy()
            er = self.ep_return[idx].cpu().numpy()
            el = self.ep_len[idx].cpu().numpy()
            ts = self.terminal_scores[idx].cpu().numpy()
            now = time.time()
            for j, i in enumerate(idx):
                term[i] = (tobs[j], er[j], el[j], ts[j])
                self.ep_score_history[i].append(list(ts[j]))
        for i in range(self.num_envs):
            info = {"scores": list(sc[i]), "play_time": float(pt[i]), "conveyor_speed": np.array([cs[i]]),
                    "out_of_reach": bool(oor[i]), "force_terminate": bool(ft[i]), "TimeLimit.truncated": False}
            if i in term:
                tobs, er, el, ts = term[i]
                info["terminal_observation"] = tobs
                info["episode"] = {"r": round(float(er), 6), "l": int(el), "t": round(now - self._t0[i], 6)}
                info["scores"] = list(ts)
                self._t0[i] = now
            infos.append(info)
        return infos

    # ------------------------------------------------------------------ SB3 VecEnv helpers
    def get_attr(self, name, indices=None):
        idx = range(self.num_envs) if indices is None else indices
        if name == "ep_score_history":
            return [self.ep_score_history[i] for i in idx]
        if name in ("num_arms", "max_num_objects", "seed"):
            return [self.env_kwargs[name] for _ in idx]
        raise AttributeError(name)

    def set_attr(self, name, value, indices=None):
        raise AttributeError(f"{name} is fixed at creation on the GPU path")

    def env_method(self, method_name, *args, indices=None, **kwargs):
        if method_name == "reset":
            n = self.num_envs
            mask = np.zeros(n, np.uint8)
            mask[list(range(n)) if indices is None else indices] = 1
            self.reset(mask=mask)
            return [None] * int(mask.sum())
        raise AttributeError(method_name)

    # ------------------------------------------------------------------ rendering (rendering.py, base_env.py:288)
    def render_tensors(self, indices=None, width=480, height=480, camera=None, frames=False):
        """Ray-cast the arenas `indices` (default: all) at their current state on the GPU (fm_render).

        Returns a uint8 tensor [len(indices), height, width, 3] on the env's device (rgb_array layout) and,
        with frames=True, the float [len(indices), ngeom, 20] geometry table it was cast from.  camera =
        (lookat_x, lookat_y, lookat_z, distance, azimuth_deg, elevation_deg) or None for the reference
        viewer's initial camera."""
        torch = self.torch
        self._bind_stream()
        idx = np.ascontiguousarray(range(self.num_envs) if indices is None else indices, dtype=np.int32).reshape(-1)
        img = torch.empty(len(idx), height, width, 3, dtype=torch.uint8, device=self.device)
        fr = None
        if frames:
            fr = torch.empty(len(idx), self._L.fm_render_ngeom(self._h), 20, dtype=torch.float32, device=self.device)
        cam = None if camera is None else (C.c_float * 6)(*[float(x) for x in camera])
        _lib.check(self._L.fm_render(self._h, idx.ctypes.data_as(C.POINTER(C.c_int32)), len(idx), int(width),
                                     int(height), cam, C.c_void_p(img.data_ptr()),
                                     C.c_void_p(fr.data_ptr()) if fr is not None else None))
        return (img, fr) if frames else img

    def get_images(self, indices=None, width=480, height=480, camera=None):
        """SB3 VecEnv.get_images: one rgb_array per env (numpy uint8 [H, W, 3])."""
        img = self.render_tensors(indices, width, height, camera).cpu().numpy()
        return list(img)

    def render(self, mode="rgb_array", indices=None, width=480, height=480, camera=None):
        """SB3 VecEnv.render("rgb_array"): the images of `indices` (default: up to the first 16 envs) tiled in a
        grid, as SB3's tile_images does."""
        if mode != "rgb_array":
            raise NotImplementedError("only rgb_array rendering (the human viewer is out of scope)")
        if indices is None:
            indices = range(min(self.num_envs, 16))
        imgs = np.stack(self.get_images(indices, width, height, camera))
        n = len(imgs)
        cols = int(np.ceil(np.sqrt(n)))
        rows = int(np.ceil(n / cols))
        pad = np.zeros((rows * cols - n,) + imgs.shape[1:], dtype=imgs.dtype)
        grid = np.concatenate([imgs, pad]).reshape(rows, cols, height, width, 3)
        return grid.transpose(0, 2, 1, 3, 4).reshape(rows * height, cols * width, 3)

    def seed(self, seed=None):
        """SB3 VecEnv.seed: per-env seeds seed + i for the next reset.  In the reference they reach
        BaseEnv.reset_sim -> gymnasium's Env.reset(seed) (base_env.py:182), which seeds only gymnasium's
        np_random; the scene (cube sizes) and the TaskManager RNG are seeded once at construction
        (base_env.py:53, task_utils.py:19) and reset never reseeds them -- so, as there, the seeds recorded here
        change no arena's trajectory (the per-arena seeds are fixed by fm_create)."""
        if seed is None:
            return [None] * self.num_envs
        self._seeds = [int(seed) + i for i in range(self.num_envs)]
        return list(self._seeds)

    def sync(self):
        _lib.check(self._L.fm_sync(self._h))

    # ------------------------------------------------------------------ state / diagnostics
    def state_size(self):
        return self._L.fm_state_size(self._h)

    def get_state(self):
        self._bind_stream()
        buf = np.zeros(self.num_envs * self.state_size(), np.uint8)
        _lib.check(self._L.fm_get_state(self._h, buf.ctypes.data_as(C.c_void_p)))
        return buf.reshape(self.num_envs, -1)

    def set_state(self, buf):
        self._bind_stream()
        self.torch.cuda.synchronize(self.device)
        buf = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
        _lib.check(self._L.fm_set_state(self._h, buf.ctypes.data_as(C.c_void_p)))

    def counters(self):
        self._bind_stream()
        out = np.zeros((self.num_envs, 8), np.int64)
        _lib.check(self._L.fm_get_counters(self._h, out.ctypes.data_as(C.c_void_p)))
        return out

    PHASES = ["fk", "geoms_mass", "collision", "rows", "smooth_acc", "newton_setup", "newton_grad",
              "newton_hessian", "newton_chol", "newton_solve", "newton_linesearch", "newton_final",
              "integrate", "task_obs"]

    def profile(self, mode=-1):
        """diagnostic phase profile (fm_profile): mode 1 zero+enable, 0 disable; returns
        ({phase: seconds summed over arenas}, ncon summed over stages)"""
        self._bind_stream()
        out = np.zeros(16, np.uint64)
        _lib.check(self._L.fm_profile(self._h, int(mode), out.ctypes.data_as(C.c_void_p)))
        khz = float(out[15]) or 1.0
        return {p: float(out[i]) / (khz * 1e3) for i, p in enumerate(self.PHASES)}, int(out[14])

    def debug_dump(self, arena=0, actuated=True):
        """diagnostic: internals of one recomputed physics stage (see fm_debug_dump)"""
        A, nv = self.env_kwargs["num_arms"], self._L.fm_nv(self._h)
        buf = np.zeros(200000)
        n = self._L.fm_debug_dump(self._h, arena, int(actuated), buf.ctypes.data_as(C.c_void_p), len(buf))
        if n < 0:
            _lib.check(n)
        out = {}
        o = 0

        def take(name, k):
            nonlocal o
            out[name] = buf[o:o + k].copy()
            o += k

        take("n", 2)
        take("Marm", 81 * A)
        take("pb", nv)
        take("as", nv)
        take("a", nv)
        take("fc", nv)
        take("site", 3 * A)
        take("bpos", 30 * A)
        take("bcom", 30 * A)
        take("dax", 27 * A)
        take("con", 17 * 64)
        take("rows", 6 * 20 * A)
        out["ncon"], out["nrow"] = int(out["n"][0]), int(out["n"][1])
        out["con"] = out["con"].reshape(64, 17)[:out["ncon"]]
        out["rows"] = out["rows"].reshape(-1, 6)[:out["nrow"]]
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._L.fm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
