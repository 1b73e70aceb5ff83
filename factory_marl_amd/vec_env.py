"""FactoryVecEnv: the SB3 VecEnv surface over N arenas resident on one MI355X.

Replaces ``make_vec_env(lambda: Monitor(Env(**env_kwargs)), n_envs, vec_env_cls=SubprocVecEnv)``
(/root/reference/src/learning.py:98-100): same ``num_envs / observation_space / action_space /
reset() / step_async() / step_wait() / step() / get_attr / set_attr / env_method / close / seed``
surface and the same auto-reset + ``infos[i]["terminal_observation"]`` + Monitor
``infos[i]["episode"] = {"r", "l", "t"}`` semantics, but every arena lives in HBM and one HIP launch
advances all of them (no worker processes, no pickled pipes).

As SB3: ``reset()`` / ``step()`` return numpy arrays.  ``return_numpy=False`` returns the torch ROCm tensors
instead, and ``step_tensors()`` is the zero-copy device path the on-GPU trainer (ppo.py) uses.

Construction: ``FactoryVecEnv(num_envs, env_class=..., env_kwargs=...)``, or SB3's ``VecEnv(env_fns)`` form -- a
list of thunks returning ``factory_marl_amd.environments`` specs, which is what ``make_vec_env(...,
vec_env_cls=FactoryVecEnv)`` passes (see environments.py).  Keyword arguments are resolved exactly as the reference
constructors resolve them (``environments.resolve_kwargs``: required ProgressRewardEnv factors, base_reward 0.0,
TypeError on unknown keywords).
"""
import ctypes as C
import math
import time

import numpy as np

from . import _lib
from . import environments as envs

# the env classes of src/environments.py with a GPU env-step (class hierarchy at environments.py:10-22)
ENV_CLASSES = {
    "FactoryManipulationEnv": _lib.FM_ENV_FACTORY,
    "AllFullRLProgressRewardEnv": _lib.FM_ENV_ALLFULLRL_PROGRESS,
    "SingleFullRLProgressRewardEnv": _lib.FM_ENV_SINGLEFULLRL_PROGRESS,
    "SingleDeltaProgressRewardEnv": _lib.FM_ENV_SINGLEDELTA_PROGRESS,
    "AllDeltaProgressRewardEnv": _lib.FM_ENV_ALLDELTA_PROGRESS,
    "PauseIKToggleEnv": _lib.FM_ENV_PAUSE_IK_TOGGLE,
    "BackupIKToggleEnv": _lib.FM_ENV_BACKUP_IK_TOGGLE,
}
TOGGLE_CLASSES = envs.TOGGLE_CLASSES

# env attributes with a value on the GPU path (base_env.py:133-147, environments.py:276-282):
# the experiment build's switches (libfactorysim_exp.so, fm_api.hip read_experiment_flags; the product library has
# none): (environment variable, value) -> flag bit.  The reference forms of the kernel's exact reformulations (the
# equivalence tests) and the rerun path's test hooks
EXPERIMENT_FLAGS = {("FM_CHOL_LDS", "2"): 2, ("FM_SERIAL_BOXBOX", "1"): 4, ("FM_NO_MIDCACHE", "1"): 8,
                    ("FM_NO_ARROW", "1"): 16, ("FM_FORCE_RERUN", "1"): 512, ("FM_NO_RERUN", "1"): 1024,
                    ("FM_NO_TREEBLK", "1"): 2048, ("FM_RERUN_AT_50", "1"): 16384}

# global scalars of the handle (fm_set_param), per-arena values of the state record, fixed at creation
RUNTIME_PARAMS = ("pt_time", "initial_conveyor_speed", "conveyor_acceleration", "force_contact_threshold",
                  "spawn_freq_increase", "init_spawn_freq", "gripper_to_closest_cube_reward_factor",
                  "closest_cube_to_bucket_reward_factor", "small_action_norm_reward_factor", "base_reward")
ARENA_SCALARS = ("play_time", "conveyor_speed")
FIXED_ATTRS = ("num_arms", "max_num_objects", "seed", "control_frequency", "frame_skip", "dt")


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


def _specs_from_env_fns(env_fns):
    """SB3 VecEnv(env_fns): every thunk must build the same env (class and keywords), as SubprocVecEnv workers of
    one make_vec_env do"""
    specs = [fn() for fn in env_fns]
    for s in specs:
        if not isinstance(s, envs.EnvSpec):
            raise TypeError("FactoryVecEnv(env_fns): the thunks must build factory_marl_amd.environments classes "
                            f"(got {type(s).__name__})")
    if any(s != specs[0] for s in specs[1:]):
        raise ValueError("FactoryVecEnv(env_fns): every env of one batch must have the same class and keywords")
    return specs[0]


class FactoryVecEnv:
    def __init__(self, num_envs, env_class="AllFullRLProgressRewardEnv", env_kwargs=None, device=0,
                 precision="fp32", seeds=None, return_numpy=True, max_contacts=0, solver_tolerance=0.0,
                 solver_iterations=0, obs_dtype=None, experimental=False):
        import torch

        self.torch = torch
        if isinstance(num_envs, (list, tuple)):  # SB3 VecEnv(env_fns) (make_vec_env(..., vec_env_cls=FactoryVecEnv))
            spec = _specs_from_env_fns(num_envs)
            num_envs, env_class, kw = len(num_envs), spec.env_class, dict(spec.kwargs)
        else:
            if env_class not in ENV_CLASSES:
                raise ValueError(f"env_class {env_class!r} not implemented on the GPU path; "
                                 f"available: {sorted(ENV_CLASSES)}")
            kw = envs.resolve_kwargs(env_class, env_kwargs or {})
        if env_class not in ENV_CLASSES:
            raise ValueError(f"env_class {env_class!r} not implemented on the GPU path; available: {sorted(ENV_CLASSES)}")
        self.env_class = env_class
        self.progress = env_class in envs.PROGRESS_CLASSES
        # experimental: the experiment build of the library (set_experiment's switches compiled in; tests / A/B only)
        L = _lib.load(experimental)
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
        # observation rows: the reference's IKTogglingEnv returns float64 rows (its float32 state columns concatenated
        # with the float64 IK proposals, environments.py:576; SubprocVecEnv stacks them as returned -- the saved
        # runs' _last_obs are float64), every other class float32.  obs_dtype overrides ("float32" / "float64").
        if obs_dtype is None:
            obs_dtype = "float64" if env_class in TOGGLE_CLASSES else "float32"
        if str(obs_dtype) not in ("float32", "float64"):
            raise ValueError(f"obs_dtype must be float32 or float64, got {obs_dtype!r}")
        cfg.obs_float64 = 1 if str(obs_dtype) == "float64" else 0
        for k in ["initial_conveyor_speed", "conveyor_acceleration", "pt_time", "force_contact_threshold",
                  "control_frequency", "spawn_freq", "spawn_freq_increase"]:
            setattr(cfg, k, float(kw[k]))
        if self.progress:  # score-reward classes have no reward factors (their kernel path reads none)
            for k in envs.PROGRESS_REQUIRED + ("base_reward",):
                setattr(cfg, k, float(kw[k]))
        if seeds is None:
            if kw["seed"] is None:
                # BaseEnv(seed=None): build_scene and the TaskManager draw fresh entropy in every env
                seeds = np.random.default_rng().integers(0, 2 ** 62, int(num_envs), dtype=np.uint64)
            else:
                seeds = [int(kw["seed"])] * int(num_envs)
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        if len(seeds) != num_envs:
            raise ValueError("need one seed per arena")
        self.seeds_used = seeds.copy()
        self.env_kwargs = kw
        # device: a GPU index / "cuda:i", or "cpu" / -1 for the CPU backend (fm_create device = -1: the kernel's own
        # sources on host threads, every buffer a CPU tensor; BASELINE config 1)
        if isinstance(device, int) and device < 0:
            device = "cpu"
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.cpu = self.device.type == "cpu"
        h = C.c_void_p()
        _lib.check(L.fm_create(C.byref(cfg), -1 if self.cpu else (self.device.index or 0),
                               seeds.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(h)), L)
        self._h = h
        self._L = L
        self.experimental = bool(experimental)
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
        odt = torch.float64 if cfg.obs_float64 else torch.float32
        self.obs_dtype = np.float64 if cfg.obs_float64 else np.float32
        self.obs = torch.zeros(n, self.obs_dim, dtype=odt, device=dev)
        self.rewards = torch.zeros(n, dtype=torch.float32, device=dev)
        self.terminated = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.scores = torch.zeros(n, 2, dtype=torch.int32, device=dev)
        self.num_obj = torch.zeros(n, dtype=torch.int32, device=dev)
        self.play_time = torch.zeros(n, dtype=torch.float64, device=dev)
        self.conveyor_speed = torch.zeros(n, dtype=torch.float64, device=dev)
        self.out_of_reach = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.force_terminate = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.terminal_obs = torch.zeros(n, self.obs_dim, dtype=odt, device=dev)
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
        self._user_attrs = [dict() for _ in range(n)]

    # ------------------------------------------------------------------ core API
    def _check(self, rc):
        _lib.check(rc, self._L)

    def _bind_stream(self):
        """run on torch's current stream so action / observation tensors are ordered with torch work"""
        if self.cpu:
            return
        s = self.torch.cuda.current_stream(self.device)
        if self._stream_bound != s.cuda_stream:
            self._check(self._L.fm_set_stream(self._h, C.c_void_p(s.cuda_stream) if s.cuda_stream else None))
            self._stream_bound = s.cuda_stream

    def reset(self, mask=None):
        self._bind_stream()
        mptr = None
        if mask is not None:
            m = self.torch.as_tensor(mask, dtype=self.torch.uint8, device=self.device).contiguous()
            mptr = C.c_void_p(m.data_ptr())
        self._check(self._L.fm_reset(self._h, mptr, C.c_void_p(self.obs.data_ptr())))
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
        self._check(self._L.fm_step(self._h, C.c_void_p(a.data_ptr()), C.c_void_p(self.obs.data_ptr()),
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
    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return [int(i) for i in indices]

    def set_experiment(self, setting=""):
        """the kernel's experiment switches on this live handle (A/B probes and equivalence tests only; a handle of the
        experiment build, FactoryVecEnv(..., experimental=True)): "FM_NO_ARROW=1 FM_NO_MIDCACHE=1" (EXPERIMENT_FLAGS)
        for the launches queued after the call; "" clears all"""
        if not self.experimental and setting:
            raise ValueError("experiment switches need the experiment build: FactoryVecEnv(..., experimental=True)")
        flags = 0
        for kv in (setting or "").split():
            k, v = kv.split("=")
            flags |= EXPERIMENT_FLAGS[(k, v)]
        self._check(self._L.fm_set_param(self._h, b"experiment_flags", float(flags)))

    def get_param(self, name):
        v = C.c_double()
        self._check(self._L.fm_get_param(self._h, name.encode(), C.byref(v)))
        return float(v.value)

    def _arena_field(self, name):
        from . import state as st

        A, K = self.env_kwargs["num_arms"], self.env_kwargs["max_num_objects"]
        return st, A, K

    def get_attr(self, name, indices=None):
        """SB3 VecEnv.get_attr: the attribute of each env in `indices`"""
        idx = self._indices(indices)
        if name == "ep_score_history":
            return [self.ep_score_history[i] for i in idx]
        if name in RUNTIME_PARAMS:
            if name in envs.PROGRESS_REQUIRED + ("base_reward",) and not self.progress:
                raise AttributeError(f"{self.env_class} has no attribute {name!r}")
            v = self.get_param(name)
            return [v for _ in idx]
        if name in ARENA_SCALARS:
            st, A, K = self._arena_field(name)
            rec = self.get_state()
            out = []
            for i in idx:
                v = float(st.fields(A, K, st.unpack(A, K, rec[i])[0])[name][0])
                out.append(np.array([v]) if name == "conveyor_speed" else v)  # base_env.py:186 keeps an array
            return out
        if name == "seed":
            return [int(self.seeds_used[i]) for i in idx]
        if name in ("num_arms", "max_num_objects", "control_frequency"):
            return [self.env_kwargs[name] for _ in idx]
        if name == "frame_skip":
            return [int((1 / self.env_kwargs["control_frequency"]) / 0.001) for _ in idx]
        if name == "dt":
            return [0.001 * int((1 / self.env_kwargs["control_frequency"]) / 0.001) for _ in idx]
        if name in ("observation_space", "action_space"):
            return [getattr(self, name) for _ in idx]
        if all(name in self._user_attrs[i] for i in idx):
            return [self._user_attrs[i][name] for i in idx]
        raise AttributeError(name)

    def set_attr(self, name, value, indices=None):
        """SB3 VecEnv.set_attr.  Runtime scalars of the env (pt_time, conveyor parameters, force threshold, spawn
        parameters, reward factors) are one value per handle: they may be set for all envs at once (or for a subset
        when the value does not change).  play_time / conveyor_speed are per-arena state.  num_arms,
        max_num_objects, seed and control_frequency fixed the compiled scene and raise.  Any other name is stored
        as a plain attribute of the envs (as setattr on the reference env would), with no effect on the step."""
        idx = self._indices(indices)
        if name in RUNTIME_PARAMS:
            v = float(np.asarray(value).reshape(-1)[0])
            # init_spawn_freq is held per arm (v / A) and read back as (v / A) * A: compare to rounding
            if len(set(idx)) != self.num_envs and not math.isclose(v, self.get_param(name), rel_tol=1e-12, abs_tol=0.0):
                raise ValueError(f"{name} is one value for all {self.num_envs} arenas of the batch: set it on every env")
            self._check(self._L.fm_set_param(self._h, name.encode(), v))
            return
        if name in ARENA_SCALARS:
            st, A, K = self._arena_field(name)
            rec = self.get_state()
            vals = np.broadcast_to(np.asarray(value, dtype=np.float64).reshape(-1), (len(idx),)) \
                if np.ndim(value) <= 1 and np.size(value) in (1, len(idx)) else None
            if vals is None:
                raise ValueError(f"{name}: one value, or one per index")
            for j, i in enumerate(idx):
                d, ints, rng = st.unpack(A, K, rec[i])
                st.fields(A, K, d)[name][0] = vals[j]
                rec[i] = st.pack(A, K, d, ints, rng)
            self.set_state(rec)
            return
        if name in FIXED_ATTRS:
            raise ValueError(f"{name} is fixed when the arenas are created (compiled scene / frame_skip / seeds)")
        for i in idx:
            self._user_attrs[i][name] = value

    # per-arena methods of the reference env with a batch-path equivalent (env_method)
    def _m_reset(self, idx, *args, **kwargs):
        n = self.num_envs
        mask = np.zeros(n, np.uint8)
        mask[idx] = 1
        obs = self.reset(mask=mask)
        obs = obs if isinstance(obs, np.ndarray) else obs.cpu().numpy()
        return [(obs[i].copy(), {}) for i in idx]  # gymnasium reset(): (obs, info)

    def _m_render(self, idx, *args, **kwargs):
        return self.get_images(idx, **kwargs)

    def _m_get_wrapper_attr(self, idx, name):
        return self.get_attr(name, idx)

    def _m_set_wrapper_attr(self, idx, name, value):
        self.set_attr(name, value, idx)
        return [None] * len(idx)

    def _m_seed(self, idx, seed=None):
        return [None if seed is None else int(seed) for _ in idx]

    def _m_close(self, idx):
        return [None] * len(idx)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        """SB3 VecEnv.env_method: call `method_name` on every env in `indices`, one result per env.  The per-arena
        methods of the reference env that exist on the batch path: reset (masked fm_reset; (obs, {}) per env),
        render (rgb_array), get_wrapper_attr / set_wrapper_attr (get_attr / set_attr), seed, close.  Methods that
        would step or rebuild one arena on its own (step, reset_sim's physics internals) have no per-arena form:
        the batch steps every arena in one launch."""
        idx = self._indices(indices)
        m = getattr(self, "_m_" + method_name, None)
        if m is None:
            raise AttributeError(f"env_method({method_name!r}): no per-arena form on the GPU path "
                                 "(available: reset, render, get_wrapper_attr, set_wrapper_attr, seed, close)")
        out = m(idx, *method_args, **method_kwargs)
        return out if isinstance(out, list) else [out] * len(idx)

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
        self._check(self._L.fm_render(self._h, idx.ctypes.data_as(C.POINTER(C.c_int32)), len(idx), int(width),
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
        self._check(self._L.fm_sync(self._h))

    # ------------------------------------------------------------------ state / diagnostics
    def state_size(self):
        return self._L.fm_state_size(self._h)

    def get_state(self):
        self._bind_stream()
        buf = np.zeros(self.num_envs * self.state_size(), np.uint8)
        self._check(self._L.fm_get_state(self._h, buf.ctypes.data_as(C.c_void_p)))
        return buf.reshape(self.num_envs, -1)

    def set_state(self, buf):
        self._bind_stream()
        if not self.cpu:
            self.torch.cuda.synchronize(self.device)
        buf = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
        self._check(self._L.fm_set_state(self._h, buf.ctypes.data_as(C.c_void_p)))

    def counters(self):
        self._bind_stream()
        out = np.zeros((self.num_envs, _lib.num_counters(self._L)), np.int64)
        self._check(self._L.fm_get_counters(self._h, out.ctypes.data_as(C.c_void_p)))
        return out

    def costs(self):
        """diagnostic: each arena's last env-step duration in GPU wall-clock ticks (fm_get_costs; the longest-first
        dispatch order is sorted by these)"""
        self._bind_stream()
        out = np.zeros(self.num_envs, np.uint32)
        self._check(self._L.fm_get_costs(self._h, out.ctypes.data_as(C.c_void_p)))
        return out

    def kernel_timing(self, enable=True):
        """time each env-step kernel launch alone (fm_kernel_timing: a HIP event pair on the env's stream around the
        step kernel; the dispatch-order kernel and the wide rerun launch stay outside)"""
        self._bind_stream()
        self._check(self._L.fm_kernel_timing(self._h, 1 if enable else 0))

    def kernel_time(self):
        """(summed milliseconds, launches) of the step-kernel launches since the last call (fm_get_kernel_time)"""
        self._bind_stream()
        ms, n = C.c_double(0.0), C.c_int(0)
        self._check(self._L.fm_get_kernel_time(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    PHASES = ["fk", "geoms_mass", "collision", "rows", "smooth_acc", "newton_setup", "newton_grad",
              "newton_hessian", "newton_chol", "newton_solve", "newton_linesearch", "newton_final",
              "integrate", "task_obs", None, None, "coll_bounds", "coll_midphase", "coll_narrow",
              "chol_diag", "chol_panel", "chol_trail", "chol_solve"]

    def profile(self, mode=-1):
        """diagnostic phase profile (fm_profile): mode 1 zero+enable, 0 disable; returns
        ({phase: seconds summed over arenas}, ncon summed over stages)"""
        self._bind_stream()
        out = np.zeros(24, np.uint64)
        self._check(self._L.fm_profile(self._h, int(mode), out.ctypes.data_as(C.c_void_p)))
        khz = float(out[15]) or 1.0
        return {p: float(out[i]) / (khz * 1e3) for i, p in enumerate(self.PHASES) if p}, int(out[14])

    def debug_dump(self, arena=0, actuated=True):
        """diagnostic: internals of one recomputed physics stage (see fm_debug_dump)"""
        A, nv = self.env_kwargs["num_arms"], self._L.fm_nv(self._h)
        buf = np.zeros(200000)
        n = self._L.fm_debug_dump(self._h, arena, int(actuated), buf.ctypes.data_as(C.c_void_p), len(buf))
        if n < 0:
            self._check(n)
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


def make_vec_env(env_id, n_envs=1, seed=None, start_index=0, monitor_dir=None, wrapper_class=None, env_kwargs=None,
                 vec_env_cls=None, vec_env_kwargs=None, monitor_kwargs=None, wrapper_kwargs=None):
    """stable_baselines3.common.env_util.make_vec_env (SB3 2.3.2 signature), building thunks of
    factory_marl_amd.environments specs: env_id is an env class (or a callable returning a spec, as learning.py's
    lambda) or a class name; vec_env_cls defaults to FactoryVecEnv.  monitor_dir / wrapper_class are not provided:
    the batch env reports the Monitor episodes itself."""
    if monitor_dir is not None or wrapper_class is not None:
        raise NotImplementedError("make_vec_env: monitor_dir / wrapper_class are not provided on the batch path")
    env_kwargs = dict(env_kwargs or {})
    if isinstance(env_id, str):
        env_id = getattr(envs, env_id)

    def make_env(rank):
        def _init():
            return env_id(**env_kwargs)
        return _init

    fns = [make_env(i + start_index) for i in range(n_envs)]
    vec = (vec_env_cls or FactoryVecEnv)(fns, **(vec_env_kwargs or {}))
    if seed is not None:
        vec.seed(seed)
    return vec
