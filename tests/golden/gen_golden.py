"""Golden-vector generator for the task layer of the env-step path.

Runs ONLY in the build container (it imports the reference from /root/reference, read-only).
It drives the reference's own Python code -- ``challenge_env/task_utils.py`` (TaskManager),
``challenge_env/base_env.py`` (BaseEnv.reset_sim/step_sim/_get_state), ``src/environments.py``
(AllFullRLProgressRewardEnv, FactoryManipulationEnv._process_action/_process_observation,
ProgressRewardEnv._get_reward) and ``challenge_env/scene.py`` (build_scene RNG draws) -- with stub
third-party modules (dm_control, gymnasium, mujoco, glfw, imageio, absl) and a *scripted* fake
physics object.  MuJoCo is absent from this image, so the fake physics does NOT
simulate: after the 100th ``physics.step()`` of an env-step it writes a pre-generated state
(qpos/qvel/site positions/contacts) into the arrays the reference reads.  Everything the reference
computes on top of that state (PCG64 spawn draws, spawn schedule, out-of-bounds / bucket scoring,
hide teleports, sort/pad, obs layout, progress reward, contact-force termination, low-pass control
targets, auto-reset) is recorded as golden data.  The fixtures are data only (npz/json); no
reference source is copied.

Usage:  python tests/golden/gen_golden.py      (writes tests/golden/*.npz, *.json)
"""
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------------------------
# stub third-party modules
# ----------------------------------------------------------------------------------------------
class _Elem:
    """Minimal stand-in for a dm_control.mjcf element (records attributes / children / attaches)."""

    def __init__(self, tag, attrs=None, parent=None):
        self.tag = tag
        self.attrs = dict(attrs or {})
        self.name = self.attrs.get("name")
        self.children = []
        self.parent = parent
        self.attached = None

    def add(self, tag, **attrs):
        e = _Elem(tag, attrs, self)
        self.children.append(e)
        return e

    def attach(self, model):
        f = _Elem("frame", {"model": model.model}, self)
        f.attached = model
        self.children.append(f)
        return f

    def set_attributes(self, **kw):
        self.attrs.update(kw)

    def _walk(self):
        yield self
        for c in self.children:
            yield from c._walk()
        if self.attached is not None:
            yield from self.attached.worldbody._walk()

    def find_all(self, tag):
        tags = {"joint": ("joint", "freejoint")}.get(tag, (tag,))
        return [e for e in self._walk() if e.tag in tags]

    def find(self, tag, name):
        for e in self._walk():
            if e.tag == tag and e.name == name:
                return e
        return _Elem(tag, {"name": name})


class _Root(_Elem):
    def __init__(self, model=None):
        super().__init__("mujoco", {"model": model})
        self.model = model
        self.worldbody = _Elem("worldbody", {}, self)

    def _walk(self):
        yield from self.worldbody._walk()

    def find_all(self, tag):
        return self.worldbody.find_all(tag)

    def find(self, tag, name):
        return self.worldbody.find(tag, name)

    def attach(self, model):
        return self.worldbody.attach(model)


SCENE_LOG = []
ENV_REF = {"env": None, "ranks": {}}


def _from_path(path):
    return _Root(model=os.path.basename(path))


def _install_stubs():
    mjcf = types.ModuleType("dm_control.mjcf")

    mjcf.RootElement = _Root
    mjcf.from_path = _from_path
    mjcf.Physics = types.SimpleNamespace(from_mjcf_model=lambda m: FakePhysics.current)
    dm = types.ModuleType("dm_control")
    dm.mjcf = mjcf
    utils = types.ModuleType("dm_control.utils")
    ik = types.ModuleType("dm_control.utils.inverse_kinematics")
    ik.qpos_from_site_pose = fake_ik
    utils.inverse_kinematics = ik
    dm.utils = utils
    sys.modules.update({"dm_control": dm, "dm_control.mjcf": mjcf, "dm_control.utils": utils,
                        "dm_control.utils.inverse_kinematics": ik})

    gym = types.ModuleType("gymnasium")

    class Env:
        def reset(self, seed=None, options=None):
            return None

    gym.Env = Env
    spaces = types.ModuleType("gymnasium.spaces")

    class Box:
        def __init__(self, low, high, dtype=np.float32, shape=None):
            self.low = np.asarray(low)
            self.high = np.asarray(high)
            self.dtype = dtype
            self.shape = self.low.shape

    class MultiDiscrete:
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec)
            self.shape = self.nvec.shape

    spaces.Box = Box
    spaces.MultiDiscrete = MultiDiscrete
    gym.spaces = spaces
    sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces})

    mj = types.ModuleType("mujoco")
    mj.viewer = types.ModuleType("mujoco.viewer")
    sys.modules.update({"mujoco": mj, "mujoco.viewer": mj.viewer})
    absl = types.ModuleType("absl")
    absl_logging = types.ModuleType("absl.logging")
    absl_logging.ERROR = 40
    absl_logging.set_verbosity = lambda v: None
    absl.logging = absl_logging
    sys.modules.update({"absl": absl, "absl.logging": absl_logging})
    # the renderer is visual-only (OUT OF SCOPE): replace the module
    rend = types.ModuleType("challenge_env.rendering")

    class MujocoRenderer:
        def __init__(self, *a, **k):
            pass

        def render(self, *a, **k):
            return None

        def close(self):
            pass

    rend.MujocoRenderer = MujocoRenderer
    sys.modules["challenge_env.rendering"] = rend


# ----------------------------------------------------------------------------------------------
# model layout (MuJoCo numbering of the compiled scene; derived in DESIGN.md §2)
# ----------------------------------------------------------------------------------------------
def layout(A, K):
    lay = {}
    lay["nq"] = 1 + 7 * K + 9 * A
    lay["nv"] = 1 + 6 * K + 9 * A
    lay["nu"] = 1 + 8 * A
    lay["ngeom"] = 13 + K + 70 * A
    q = {}
    v = {}
    q["conveyor"] = 0
    v["conveyor"] = 0
    for k in range(K):
        q[f"cube{k}"] = 1 + 7 * k
        v[f"cube{k}"] = 1 + 6 * k
    for i in range(A):
        for j in range(1, 8):
            q[f"arm{i}/iiwa14/joint{j}"] = 1 + 7 * K + 9 * i + (j - 1)
            v[f"arm{i}/iiwa14/joint{j}"] = 1 + 6 * K + 9 * i + (j - 1)
        q[f"arm{i}/iiwa14/single_gripper/left_plate_slide_joint"] = 1 + 7 * K + 9 * i + 7
        v[f"arm{i}/iiwa14/single_gripper/left_plate_slide_joint"] = 1 + 6 * K + 9 * i + 7
        q[f"arm{i}/iiwa14/single_gripper/right_plate_slide_joint"] = 1 + 7 * K + 9 * i + 8
        v[f"arm{i}/iiwa14/single_gripper/right_plate_slide_joint"] = 1 + 6 * K + 9 * i + 8
    lay["qadr"] = q
    lay["vadr"] = v
    g = {}
    for i in range(A):
        base = 13 + K + 70 * i
        for j in range(61):
            g[f"arm{i}/iiwa14//unnamed_geom_{j}"] = base + j
        for j in range(9):
            g[f"arm{i}/iiwa14/single_gripper//unnamed_geom_{j}"] = base + 61 + j
    lay["geom"] = g
    lim = [(-1.0, 1.0)]
    arm_rng = [2.96706, 2.0944, 2.96706, 2.0944, 2.96706, 2.0944, 3.05433]
    for i in range(A):
        lim += [(-r, r) for r in arm_rng] + [(0.0, 0.060000000000000005)]
    lay["ctrlrange"] = np.array(lim)
    return lay


def bucket_pos(A):
    by = 0.7 - (A // 2 - 1)
    return [np.array([0.9, by, 1.05 - 0.04]), np.array([-0.9, by, 1.05 - 0.04])]


# ----------------------------------------------------------------------------------------------
# scripted fake physics
# ----------------------------------------------------------------------------------------------
class _Binding:
    def __init__(self, phys, objs):
        self.p = phys
        self.objs = objs

    def _idx(self, which):
        lst = self.objs if isinstance(self.objs, list) else [self.objs]
        out = []
        for o in lst:
            k = int(o.parent.attrs["model"].replace("cube", "")) if o.tag == "freejoint" else None
            if which == "q":
                out += list(range(1 + 7 * k, 8 + 7 * k))
            else:
                out += list(range(1 + 6 * k, 7 + 6 * k))
        return np.array(out, dtype=np.int64)

    @property
    def qpos(self):
        return _View(self.p.data.qpos, self._idx("q"))

    @qpos.setter
    def qpos(self, val):
        self.p.data.qpos[self._idx("q")] = val

    @property
    def qvel(self):
        return _View(self.p.data.qvel, self._idx("v"))

    @qvel.setter
    def qvel(self, val):
        self.p.data.qvel[self._idx("v")] = val

    @property
    def xpos(self):
        return self.p.bucket_xpos[self.objs.attrs["_bucket"]].copy()

    @property
    def size(self):
        return np.array([0.29, 0.29, 0.02])


class _View:
    def __init__(self, arr, idx):
        self.arr = arr
        self.idx = idx

    def __getitem__(self, key):
        return self.arr[self.idx][key]

    def __setitem__(self, key, val):
        tmp = self.arr[self.idx]
        tmp[key] = val
        self.arr[self.idx] = tmp

    def copy(self):
        return self.arr[self.idx].copy()

    def reshape(self, *s):
        return self.arr[self.idx].reshape(*s)

    def __array__(self, dtype=None, copy=None):
        a = self.arr[self.idx]
        return a.astype(dtype) if dtype is not None else a


class _Named:
    def __init__(self, phys):
        self.p = phys
        lay = phys.lay

        class QI:
            def __init__(s, arr, adr):
                s.arr, s.adr = arr, adr

            def __getitem__(s, names):
                if isinstance(names, str):
                    return s.arr[s.adr[names]]
                return s.arr[[s.adr[n] for n in names]]

        class SI:
            def __getitem__(s, name):
                return phys.sites[name]

        self.data = types.SimpleNamespace(qpos=QI(phys.data.qpos, lay["qadr"]),
                                          qvel=QI(phys.data.qvel, lay["vadr"]), site_xpos=SI())


class _Contacts:
    def __init__(self, geoms):
        self.geom = np.array(geoms, dtype=np.int32).reshape(-1, 2)


class FakePhysics:
    current = None

    def __init__(self, A, K, script):
        self.A, self.K = A, K
        self.lay = layout(A, K)
        self.script = script
        nq, nv, nu = self.lay["nq"], self.lay["nv"], self.lay["nu"]
        self.model = types.SimpleNamespace(
            opt=types.SimpleNamespace(timestep=0.001), actuator_ctrlrange=self.lay["ctrlrange"].copy(),
            nu=nu, _model=types.SimpleNamespace(vis=types.SimpleNamespace(global_=types.SimpleNamespace())),
            name2id=self._name2id)
        self.data = types.SimpleNamespace(qpos=np.zeros(nq), qvel=np.zeros(nv), ctrl=np.zeros(nu), ncon=0,
                                          contact=_Contacts([]), contact_force=self._contact_force, _data=None)
        self.sites = {}
        for i in range(A):
            xi = 0.7 * (-1) ** i
            yi = 1.4 * (i // 2) - (A // 2 - 1)
            self.sites[f"arm{i}/player_site"] = np.array([xi, yi, 1.0])
            self.sites[f"arm{i}/iiwa14/single_gripper/between_gripper_plates"] = np.array([xi, yi, 2.3])
        self.bucket_xpos = bucket_pos(A)
        self.forces = []
        self.named = _Named(self)
        self.nstep = 0
        self.ctrl_log = []

    def _name2id(self, name, kind):
        if kind == "geom":
            return self.lay["geom"][name]
        if kind == "joint":
            return self.lay["qadr"][name]
        raise KeyError(name)

    def _contact_force(self, i):
        return self.forces[i].copy()

    def bind(self, obj):
        return _Binding(self, obj)

    def reset(self):
        self.data.qpos[:] = 0.0
        self.data.qvel[:] = 0.0
        self.data.qpos[[1 + 7 * k + 3 for k in range(self.K)]] = 1.0  # free-joint qpos0 quaternion
        self.data.ncon = 0
        self.data.contact = _Contacts([])
        self.forces = []

    def after_reset(self):
        pass

    def get_state(self):
        return np.concatenate([self.data.qpos, self.data.qvel])

    def set_control(self, ctrl):
        self._last_ctrl = np.array(ctrl, dtype=np.float64)
        self.ctrl_log.append(self._last_ctrl.copy())

    def step(self):
        self.nstep += 1
        if self.nstep % 100 == 0:
            self.script(self)

    def copy(self, share_model=True):
        # physics.copy(share_model=True) (ik_policy.py:270): a separate data block, the model shared
        return _PhysicsCopy(self)


class _PhysicsCopy:
    def __init__(self, p):
        self.lay = p.lay
        self.data = types.SimpleNamespace(qpos=p.data.qpos.copy(), qvel=p.data.qvel.copy())
        lay = p.lay
        data = self.data

        class QI:
            def __getitem__(s, names):
                if isinstance(names, str):
                    return data.qpos[lay["qadr"][names]]
                return data.qpos[[lay["qadr"][n] for n in names]]

        self.named = types.SimpleNamespace(data=types.SimpleNamespace(qpos=QI()))


FAKE_IK_CALLS = []


def fake_ik(physics, site, target_pos, target_quat, joint_names, max_steps=10):
    # deterministic, non-physical stand-in for dm_control IK (IK numerics are parity-unpinned); the
    # success flag varies with the target so both branches of ik_policy.py:266-282 are exercised
    q = np.zeros(physics.lay["nq"])
    for n, j in enumerate(joint_names):
        q[physics.lay["qadr"][j]] = np.tanh(target_pos[n % 3] + 0.1 * n)
    ok = bool(target_pos[2] < 5.0) and int(abs(float(target_pos[0])) * 1e4) % 5 != 0
    arm = int(site.split("/")[0].replace("arm", ""))
    FAKE_IK_CALLS.append(dict(arm=arm, target_pos=np.array(target_pos, dtype=np.float64),
                              target_quat=np.array(target_quat, dtype=np.float64), success=ok,
                              q7=np.array([q[physics.lay["qadr"][j]] for j in joint_names])))
    return types.SimpleNamespace(success=ok, qpos=q, steps=1)


# ----------------------------------------------------------------------------------------------
# scripts: what the fake "physics" puts into the state at the end of each env-step
# ----------------------------------------------------------------------------------------------
def make_script(rng, A, K, lay, events):
    arm_rng = np.array([2.96706, 2.0944, 2.96706, 2.0944, 2.96706, 2.0944, 3.05433])
    bpos = bucket_pos(A)
    step = {"n": 0}

    def script(p):
        step["n"] += 1
        n = step["n"]
        tm = ENV_REF["env"].task_manager
        ENV_REF["ranks"] = {int(o.parent.attrs["model"].replace("cube", "")): r for r, o in enumerate(tm._in_scene)}
        q, v = p.data.qpos, p.data.qvel
        # arms
        for i in range(A):
            a = 1 + 7 * K + 9 * i
            b = 1 + 6 * K + 9 * i
            q[a:a + 7] = rng.uniform(-1, 1, 7) * arm_rng
            q[a + 7:a + 9] = rng.uniform(-0.002, 0.062, 2)
            v[b:b + 9] = rng.normal(0, 0.5, 9)
            p.sites[f"arm{i}/iiwa14/single_gripper/between_gripper_plates"] = (
                p.sites[f"arm{i}/player_site"] + rng.uniform(-0.8, 0.8, 3) * np.array([1, 1, 0.6])
                + np.array([0, 0, 0.5]))
        q[0] -= 0.01
        v[0] = -0.1
        ev = events.get(n, {})
        for k in range(K):
            a = 1 + 7 * k
            b = 1 + 6 * k
            x, y, z = q[a:a + 3]
            if x >= 3.0:  # parked / hidden cube: let it rest on the floor
                q[a + 2] = 0.04
                v[b:b + 6] = 0.0
                continue
            if z > 1.5:  # just spawned: land on the belt
                q[a:a + 3] = [rng.normal(0, 0.05), 1.0 - rng.uniform(0, 0.05), 1.13 + rng.uniform(0, 0.01)]
            else:
                q[a + 1] -= rng.uniform(0.005, 0.02)
                q[a] += rng.normal(0, 0.01)
            qq = rng.normal(0, 1, 4)
            q[a + 3:a + 7] = qq / np.linalg.norm(qq)
            v[b:b + 6] = rng.normal(0, 0.1, 6)
            rank = ENV_REF["ranks"].get(k)
            if ev.get("need", 0) > len(ENV_REF["ranks"]):
                ev = {}
            for (kk, bi, kind) in ev.get("bucket", []):
                if kk != rank:
                    continue
                c = bpos[bi]
                off = {"in": [0.0, 0.0, 0.07], "edge_x": [0.6 * 0.29, 0.0, 0.05],
                       "out_x": [0.6 * 0.29 + 1e-9, 0.0, 0.05], "high": [0.0, 0.0, 0.0800001],
                       "edge_z": [0.0, -0.6 * 0.29, 0.01 + 0.07], "corner": [-0.174, 0.174, 0.02]}[kind]
                q[a:a + 3] = c + np.array(off)
            for (kk, kind) in ev.get("oob", []):
                if kk != rank:
                    continue
                if kind == "x":
                    q[a] = 1.2000001
                elif kind == "x_edge":
                    q[a] = -1.2
                elif kind == "y":
                    q[a + 1] = -1.5000001
                elif kind == "y_edge":
                    q[a + 1] = -1.5
                elif kind == "z":
                    q[a + 2] = 0.8999999
                elif kind == "z_edge":
                    q[a + 2] = 0.9
            if ev.get("tie") and rank is not None and rank < 2:
                q[a] = 0.125
        # contacts
        geoms, forces = [], []
        nc = rng.integers(0, 6)
        for c in range(nc):
            g1 = int(rng.integers(0, lay["ngeom"]))
            g2 = int(rng.integers(0, lay["ngeom"]))
            geoms.append((min(g1, g2), max(g1, g2)))
            forces.append(rng.normal(0, 40, 6))
        if "force" in ev:
            arm_g = 13 + K + 70 * ev["force"][0] + 30
            geoms.append((3, arm_g))
            f = np.zeros(6)
            f[ev["force"][1]] = ev["force"][2]
            forces.append(f)
        if "force_nonarm" in ev:
            geoms.append((1, 3))
            forces.append(np.array([500.0, 0, 0, 0, 0, 0]))
        p.data.ncon = len(geoms)
        p.data.contact = _Contacts(geoms)
        p.forces = forces

    return script


def gen_episodes(env_cls_name, A, K, seed, n_steps, events, reward_kw, tag, act_seed=0):
    import environments as envs_mod

    rng = np.random.default_rng(1000 + seed + 17 * A + K)
    lay = layout(A, K)
    script = make_script(rng, A, K, lay, events)
    FakePhysics.current = FakePhysics(A, K, script)
    cls = getattr(envs_mod, env_cls_name)
    kw = dict(num_arms=A, max_num_objects=K, seed=seed, render_mode="rgb_array")
    kw.update(reward_kw)
    env = cls(**kw)
    ENV_REF["env"] = env
    phys = FakePhysics.current
    arng = np.random.default_rng(act_seed)
    rec = {k: [] for k in ["action", "obs", "reward", "terminated", "scores", "play_time", "conveyor_speed",
                           "out_of_reach", "force_terminate", "pre_qpos", "pre_qvel", "post_qpos", "post_qvel",
                           "ncon", "con_geom", "con_force", "grip_site", "ctrl_samples", "num_obj",
                           "reset_after", "in_scene", "spawn_freq", "step_counter"]}
    obs, _ = env.reset()
    rec["obs0"] = obs.copy()
    rec["obs_dtype"] = str(obs.dtype)
    maxc = 12
    for t in range(n_steps):
        if env_cls_name.endswith("ToggleEnv"):
            action = arng.integers(0, 2, A)
        else:
            action = arng.uniform(-3, 3, 8 * A).astype(np.float32)
        phys.ctrl_log = []
        # capture pre-task physics state: the script fires inside the 100th physics.step()
        orig_tm_step = env.task_manager.step

        def tm_step_wrap():
            rec["pre_qpos"].append(phys.data.qpos.copy())
            rec["pre_qvel"].append(phys.data.qvel.copy())
            orig_tm_step()

        env.task_manager.step = tm_step_wrap
        obs, reward, term, trunc, info = env.step(action)
        env.task_manager.step = orig_tm_step
        rec["action"].append(np.asarray(action).astype(np.float32) if action.dtype != np.int64 else action)
        rec["obs"].append(obs.copy())
        rec["reward"].append(float(reward))
        rec["terminated"].append(bool(term))
        rec["scores"].append(list(info["scores"]))
        rec["play_time"].append(info["play_time"])
        rec["conveyor_speed"].append(float(info["conveyor_speed"][0]))
        rec["out_of_reach"].append(bool(info["out_of_reach"]))
        rec["force_terminate"].append(bool(info["force_terminate"]))
        rec["post_qpos"].append(phys.data.qpos.copy())
        rec["post_qvel"].append(phys.data.qvel.copy())
        cg = np.full((maxc, 2), -1, np.int32)
        cf = np.zeros((maxc, 6))
        cg[:phys.data.ncon] = phys.data.contact.geom
        for c in range(phys.data.ncon):
            cf[c] = phys.forces[c]
        rec["ncon"].append(phys.data.ncon)
        rec["con_geom"].append(cg)
        rec["con_force"].append(cf)
        rec["grip_site"].append(np.stack([phys.sites[f"arm{i}/iiwa14/single_gripper/between_gripper_plates"]
                                          for i in range(A)]))
        cl = np.array(phys.ctrl_log)
        rec["ctrl_samples"].append(cl[[0, 1, 49, 99]])
        rec["num_obj"].append(len(env.task_manager._in_scene))
        ins = [int(o.parent.attrs["model"].replace("cube", "")) for o in env.task_manager._in_scene]
        rec["in_scene"].append(ins + [-1] * (K - len(ins)))
        rec["spawn_freq"].append(env.task_manager.spawn_freq)
        rec["step_counter"].append(env.task_manager._step_counter)
        if term:
            env.reset()
            rec["reset_after"].append(True)
        else:
            rec["reset_after"].append(False)
    out = {}
    for k, v in rec.items():
        if k == "obs_dtype":
            continue
        out[k] = np.asarray(v)
    out["A"] = A
    out["K"] = K
    out["seed"] = seed
    np.savez_compressed(os.path.join(OUT, f"task_{tag}.npz"), **out)
    meta = {"env_class": env_cls_name, "A": A, "K": K, "seed": seed, "n_steps": n_steps,
            "reward_kw": reward_kw, "obs_dtype": rec.get("obs_dtype"),
            "episodes": int(np.sum(out["terminated"]))}
    return meta


# ----------------------------------------------------------------------------------------------
# IK base policy episodes (ik_policy.py + the IK env classes of environments.py)
# ----------------------------------------------------------------------------------------------
IK_STATE_NAMES = ["IDLE", "GO_TO_GRASP", "GRASP_APPROACH", "GRASP_CLOSE", "POST_GRASP", "GO_TO_RELEASE", "RELEASE"]


def _cube_idx(obj):
    return -1 if obj is None else int(obj.parent.attrs["model"].replace("cube", ""))


def make_ik_script(rng, A, K, lay):
    """cooperative fake physics: arms track their last command, grippers land near their last IK target,
    grasped cubes follow the gripper, released cubes drop into the bucket -- so every FSM edge is taken"""
    arm_rng = np.array([2.96706, 2.0944, 2.96706, 2.0944, 2.96706, 2.0944, 3.05433])
    bpos = bucket_pos(A)
    step = {"n": 0}

    def script(p):
        step["n"] += 1
        env = ENV_REF["env"]
        tm = env.task_manager
        q, v = p.data.qpos, p.data.qvel
        last_target = ENV_REF.setdefault("last_target", {})
        for c in FAKE_IK_CALLS:
            last_target[c["arm"]] = c["target_pos"]
        for i in range(A):
            a = 1 + 7 * K + 9 * i
            b = 1 + 6 * K + 9 * i
            cmd = p._last_ctrl[1 + 8 * i:1 + 8 * i + 7]
            if rng.random() < 0.85:
                q[a:a + 7] = cmd + rng.normal(0, 0.03, 7)
            else:
                q[a:a + 7] = rng.uniform(-1, 1, 7) * arm_rng
            q[a + 7:a + 9] = rng.uniform(0.0, 0.06, 2)
            v[b:b + 9] = rng.normal(0, 0.3, 9)
            base = p.sites[f"arm{i}/player_site"]
            holding = env.ik_policies[i].state.name in ("GRASP_CLOSE", "POST_GRASP", "GO_TO_RELEASE")
            if i in last_target and rng.random() < (0.97 if holding else 0.85):
                site = last_target[i] + rng.normal(0, 0.015, 3)
            else:  # somewhere in the arm's workspace, inside the TaskManager bounds (|x| <= 1.2)
                site = base + rng.uniform(-0.45, 0.45, 3) * np.array([1, 1, 0.6]) + np.array([0, 0, 0.5])
            p.sites[f"arm{i}/iiwa14/single_gripper/between_gripper_plates"] = site
        q[0] -= 0.01
        v[0] = -0.1
        holders = {}
        for i, pol in enumerate(env.ik_policies):
            k = _cube_idx(pol.target_object)
            if k >= 0:
                holders[k] = (i, pol.state.name)
        for o in tm._in_scene:
            k = _cube_idx(o)
            a = 1 + 7 * k
            b = 1 + 6 * k
            if q[a + 2] > 1.5:  # just spawned: land on the belt
                q[a:a + 3] = [rng.normal(0, 0.05), 1.0 - rng.uniform(0, 0.05), 1.13 + rng.uniform(0, 0.01)]
            else:
                q[a + 1] -= rng.uniform(0.02, 0.06)
                q[a] += rng.normal(0, 0.01)
            qq = rng.normal(0, 1, 4)
            q[a + 3:a + 7] = qq / np.linalg.norm(qq)
            v[b:b + 6] = rng.normal(0, 0.1, 6)
            if k in holders:
                i, st = holders[k]
                grip = p.sites[f"arm{i}/iiwa14/single_gripper/between_gripper_plates"]
                if st in ("GRASP_APPROACH", "GRASP_CLOSE", "POST_GRASP", "GO_TO_RELEASE") and rng.random() < 0.96:
                    q[a:a + 3] = grip + rng.normal(0, 0.01, 3)
                elif st == "RELEASE" and rng.random() < 0.5:
                    q[a:a + 3] = bpos[i % 2] + np.array([0.0, 0.0, 0.05])
        geoms, forces = [], []
        if step["n"] % 97 == 0:  # an occasional force termination -> reset coverage
            geoms.append((3, 13 + K + 70 * (step["n"] % A) + 30))
            forces.append(np.array([250.0, 0, 0, 0, 0, 0]))
        p.data.ncon = len(geoms)
        p.data.contact = _Contacts(geoms)
        p.forces = forces

    return script


def gen_ik_episodes(env_cls_name, A, K, seed, n_steps, tag, act_seed=0):
    """act()-level and compose-level records of the reference's IKPolicy under a fake IK solver"""
    import environments as envs_mod
    import challenge_env.ik_policy as ikp

    rng = np.random.default_rng(2000 + seed + 17 * A + K)
    lay = layout(A, K)
    FakePhysics.current = FakePhysics(A, K, make_ik_script(rng, A, K, lay))
    phys = FakePhysics.current
    phys._last_ctrl = np.zeros(lay["nu"])
    ENV_REF.pop("last_target", None)
    acts, comps = [], []
    cur = {"step": -1, "compose": -1}

    def snap(pol):
        ign = [-1] * A
        for owner, obj in pol.ignore_objects.items():
            ign[owner] = _cube_idx(obj)
        ms = pol._move_start_pos
        return dict(state=int(pol.state.value), counter=int(pol.state_counter), target=_cube_idx(pol.target_object),
                    ignore=ign, last_ctrl=np.array(pol.last_ctrl, dtype=np.float64),
                    move_start=np.zeros(3) if ms is None else np.array(ms, dtype=np.float64))

    orig_act = ikp.IKPolicy.act

    def rec_act(self):
        env = ENV_REF["env"]
        before = snap(self)
        n0 = len(FAKE_IK_CALLS)
        out = orig_act(self)
        calls = FAKE_IK_CALLS[n0:]
        acts.append(dict(step=cur["step"], compose=cur["compose"], arm=self.arm_id, before=before, after=snap(self),
                         ctrl=np.array(out, dtype=np.float64), calls=calls))
        return out

    ikp.IKPolicy.act = rec_act
    orig_compose = envs_mod.FactoryManipulationEnv._compose_control

    def rec_compose(self, action):
        # record the IK compose: FactoryManipulationEnv's own (step passes the action) or an override's super()
        # call (passes None); AllFullRL-style overrides never get here
        if action is not None and type(self)._compose_control is not rec_compose:
            return orig_compose(self, action)
        cur["compose"] += 1
        tm = self.task_manager
        p = self.physics
        rec = dict(step=cur["step"], compose=cur["compose"], qpos=p.data.qpos.copy(), qvel=p.data.qvel.copy(),
                   grip=np.stack([p.sites[f"arm{i}/iiwa14/single_gripper/between_gripper_plates"].copy()
                                  for i in range(A)]),
                   base=np.stack([p.sites[f"arm{i}/player_site"].copy() for i in range(A)]),
                   in_scene=[_cube_idx(o) for o in tm._in_scene],
                   before=[snap(pol) for pol in self.ik_policies])
        out = orig_compose(self, action)
        rec["after"] = [snap(pol) for pol in self.ik_policies]
        rec["arm_ctrl"] = np.concatenate([np.asarray(x, dtype=np.float64) for x in out])
        comps.append(rec)
        return out

    envs_mod.FactoryManipulationEnv._compose_control = rec_compose
    cls = getattr(envs_mod, env_cls_name)
    prog = dict(gripper_to_closest_cube_reward_factor=0.2, closest_cube_to_bucket_reward_factor=0.4,
                small_action_norm_reward_factor=0.3, base_reward=0.4)
    kw = dict(num_arms=A, max_num_objects=K, seed=seed, render_mode="rgb_array")
    if issubclass(cls, envs_mod.ProgressRewardEnv):
        kw.update(prog)
    env = cls(**kw)
    ENV_REF["env"] = env
    orig_set = phys.set_control

    def set_control(ctrl):
        orig_set(ctrl)
        phys._last_ctrl = np.array(ctrl, dtype=np.float64)

    phys.set_control = set_control
    sent = []
    orig_unscaled = env._step_sim_unscaled

    def rec_unscaled(ctrl):
        sent.append(np.array(ctrl, dtype=np.float64))
        return orig_unscaled(ctrl)

    env._step_sim_unscaled = rec_unscaled
    arng = np.random.default_rng(act_seed)
    steps = []
    obs, _ = env.reset()
    obs0 = np.asarray(obs, dtype=np.float64)
    for t in range(n_steps):
        cur["step"] = t
        if env_cls_name.endswith("ToggleEnv"):
            action = arng.integers(0, 2, A)
        else:
            action = arng.uniform(-2, 2, env.action_space.shape[0]).astype(np.float32)
        obs, reward, term, trunc, info = env.step(action)
        steps.append(dict(action=np.asarray(action, dtype=np.float64), obs=np.asarray(obs, dtype=np.float64),
                          reward=float(reward), terminated=bool(term), scores=list(info["scores"]),
                          sent=sent[-1][1:].copy(), post_qpos=phys.data.qpos.copy(),
                          post_grip=np.stack([phys.sites[f"arm{i}/iiwa14/single_gripper/between_gripper_plates"].copy()
                                              for i in range(A)]),
                          post_in_scene=[_cube_idx(o) for o in env.task_manager._in_scene] +
                          [-1] * (K - len(env.task_manager._in_scene))))
        if term:
            cur["step"] = t + 0.5
            env.reset()
    ikp.IKPolicy.act = orig_act
    envs_mod.FactoryManipulationEnv._compose_control = orig_compose
    # flatten to arrays
    out = {"A": A, "K": K, "seed": seed, "obs0": obs0}
    for key in ["action", "obs", "reward", "terminated", "scores", "sent", "post_qpos", "post_grip", "post_in_scene"]:
        out[f"step_{key}"] = np.asarray([s[key] for s in steps])
    def arm_arrays(prefix, recs):
        out[f"{prefix}_i"] = np.asarray([[r["state"], r["counter"], r["target"]] + r["ignore"] for r in recs], np.int32)
        out[f"{prefix}_d"] = np.asarray([np.concatenate([r["last_ctrl"], r["move_start"]]) for r in recs])
    arm_arrays("act_before", [a["before"] for a in acts])
    arm_arrays("act_after", [a["after"] for a in acts])
    out["act_meta"] = np.asarray([[a["step"] * 2, a["compose"], a["arm"], len(a["calls"])] for a in acts], np.int64)
    out["act_ctrl"] = np.asarray([a["ctrl"] for a in acts])
    out["act_call_args"] = np.asarray([np.concatenate([a["calls"][0]["target_pos"], a["calls"][0]["target_quat"]])
                                       if a["calls"] else np.full(7, np.nan) for a in acts])
    out["act_call_result"] = np.asarray([np.concatenate([[float(a["calls"][0]["success"])], a["calls"][0]["q7"]])
                                         if a["calls"] else np.full(8, np.nan) for a in acts])
    # inputs of each act = its compose's physics snapshot
    out["comp_meta"] = np.asarray([[c["step"] * 2, c["compose"], len(c["in_scene"])] for c in comps], np.int64)
    out["comp_qpos"] = np.asarray([c["qpos"] for c in comps])
    out["comp_qvel"] = np.asarray([c["qvel"] for c in comps])
    out["comp_grip"] = np.asarray([c["grip"] for c in comps])
    out["comp_base"] = np.asarray([c["base"] for c in comps])
    out["comp_in_scene"] = np.asarray([c["in_scene"] + [-1] * (K - len(c["in_scene"])) for c in comps], np.int32)
    out["comp_arm_ctrl"] = np.asarray([c["arm_ctrl"] for c in comps])
    for which in ["before", "after"]:
        recs = [r for c in comps for r in c[which]]
        out[f"comp_{which}_i"] = np.asarray([[r["state"], r["counter"], r["target"]] + r["ignore"] for r in recs],
                                            np.int32).reshape(len(comps), A, -1)
        out[f"comp_{which}_d"] = np.asarray([np.concatenate([r["last_ctrl"], r["move_start"]]) for r in recs]
                                            ).reshape(len(comps), A, -1)
    np.savez_compressed(os.path.join(OUT, f"ik_{tag}.npz"), **out)
    hist = {}
    for a in acts:
        n = IK_STATE_NAMES[a["after"]["state"]]
        hist[n] = hist.get(n, 0) + 1
    return {"env_class": env_cls_name, "A": A, "K": K, "seed": seed, "n_steps": n_steps, "acts": len(acts),
            "composes": len(comps), "ik_calls": int(sum(len(a["calls"]) for a in acts)),
            "ik_success": int(sum(c["success"] for a in acts for c in a["calls"])),
            "episodes": int(sum(s["terminated"] for s in steps)), "states_after_act": hist,
            "scores_final": steps[-1]["scores"]}


def gen_rng_vectors():
    """PCG64/SeedSequence draws as the reference consumes them (scene.py:121-131, task_utils.py:47-52)."""
    out = {}
    for seed in [0, 1, 42, 12345, 2**40 + 7]:
        r = np.random.default_rng(seed)
        out[f"uniform_{seed}"] = r.uniform(0, 1, 64)
        bg = np.random.PCG64(seed)
        st = bg.state["state"]
        out[f"state_{seed}"] = np.array([st["state"] >> 64, st["state"] & (2**64 - 1),
                                         st["inc"] >> 64, st["inc"] & (2**64 - 1)], dtype=np.uint64)
    return out


def gen_scene_draws():
    """Cube half-sizes drawn by build_scene (scene.py:121-131) and the arm/bucket placement it records."""
    import challenge_env.scene as scene

    res = {}
    for A, K, seed in [(2, 4, 42), (2, 8, 42), (4, 16, 42), (2, 10, 42), (2, 4, 7), (4, 10, 3)]:
        sizes = []
        orig = scene.PickableObject

        class Rec(orig):
            def __init__(self, name, size=0.04, color=None):
                sizes.append(size)
                super().__init__(name, size=size, color=color)

        scene.PickableObject = Rec
        arms = []
        orig_arm = scene.Arm

        class RecArm(orig_arm):
            def __init__(self, pos, name, flip=False, mount_ceiling=False):
                arms.append((list(map(float, pos)), bool(flip)))
                super().__init__(pos, name, flip, mount_ceiling)

        scene.Arm = RecArm
        root = scene.build_scene(num_objects=K, seed=seed, num_arms=A)
        scene.PickableObject = orig
        scene.Arm = orig_arm
        geoms = [e for e in root.find_all("geom")]
        tables = [g.attrs for g in geoms if g.attrs.get("name") == "table"]
        buckets = [e.attrs for e in root.find_all("body") if e.attrs.get("name") == "bucket"]
        res[f"{A}_{K}_{seed}"] = {
            "sizes": [float(s) for s in sizes],
            "masses": [float(1000 * s ** 3) for s in sizes],
            "arms": arms,
            "table_size": [float(x) for x in tables[0]["size"]],
            "bucket_pos": [[float(x) for x in b["pos"]] for b in buckets],
        }
    return res


def main_ik():
    """IK fixtures only (ik_*.npz + ik_meta.json); the task-layer fixtures stay as they are"""
    meta = {"generator": "tests/golden/gen_golden.py --ik", "reference": "nkirschi/Factory-MARL @ 2024-12-20",
            "numpy": np.__version__, "fixtures": {}}
    for cls, A, K, seed, n, tag, aseed in [("FactoryManipulationEnv", 2, 4, 42, 400, "factory_2x4", 0),
                                           ("PauseIKToggleEnv", 4, 16, 42, 300, "pause_4x16", 1),
                                           ("BackupIKToggleEnv", 2, 8, 7, 300, "backup_2x8", 2),
                                           ("SingleDeltaProgressRewardEnv", 2, 4, 42, 300, "singledelta_2x4", 3),
                                           ("AllDeltaProgressRewardEnv", 2, 6, 5, 300, "alldelta_2x6", 4),
                                           ("SingleFullRLProgressRewardEnv", 2, 4, 9, 300, "singlefull_2x4", 5)]:
        meta["fixtures"][tag] = gen_ik_episodes(cls, A, K, seed, n, tag, act_seed=aseed)
        print(tag, json.dumps(meta["fixtures"][tag]))
    with open(os.path.join(OUT, "ik_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


def _setup():
    sys.path.insert(0, os.path.join(REF, "challenge_env"))
    sys.path.insert(0, os.path.join(REF, "src"))
    _install_stubs()
    import challenge_env.task_utils as tu  # noqa: F401

    # bucket geoms in the fake scene carry which bucket they are
    orig_init = tu.TaskManager.__init__

    def tm_init(self, physics, mjcf_model, seed=None, spawn_freq=0.25):
        orig_init(self, physics, mjcf_model, seed=seed, spawn_freq=spawn_freq)
        for bi, b in enumerate(self.buckets):
            b.attrs["_bucket"] = bi

    tu.TaskManager.__init__ = tm_init


def main():
    _setup()
    meta = {"generator": "tests/golden/gen_golden.py", "reference": "nkirschi/Factory-MARL @ 2024-12-20",
            "numpy": np.__version__, "fixtures": {}}
    np.savez_compressed(os.path.join(OUT, "rng_pcg64.npz"), **gen_rng_vectors())
    with open(os.path.join(OUT, "scene_draws.json"), "w") as f:
        json.dump(gen_scene_draws(), f, indent=1)

    prog = dict(gripper_to_closest_cube_reward_factor=0.2, closest_cube_to_bucket_reward_factor=0.4,
                small_action_norm_reward_factor=0.3, base_reward=0.4)
    ev_a = {3: {"bucket": [(0, 0, "in")]}, 50: {"bucket": [(0, 1, "edge_x")]},
            95: {"bucket": [(0, 0, "out_x"), (1, 1, "in")]}, 100: {"tie": True},
            101: {"tie": True, "bucket": [(1, 0, "high")]},
            140: {"bucket": [(0, 1, "edge_z"), (1, 1, "in"), (2, 0, "corner")]}, 150: {"force_nonarm": True},
            160: {"force": (1, 2, 200.0)}, 170: {"oob": [(0, "x_edge")]}, 175: {"oob": [(1, "y_edge")]},
            180: {"oob": [(0, "z_edge")]}, 190: {"oob": [(1, "y")]},
            230: {"force": (0, 0, -200.0001)}, 300: {"oob": [(0, "z"), (0, "x")]},
            335: {"bucket": [(0, 0, "in"), (1, 0, "in")]}, 380: {"oob": [(0, "x")]}}
    meta["fixtures"]["fullrl_2x4"] = gen_episodes("AllFullRLProgressRewardEnv", 2, 4, 42, 420, ev_a, prog,
                                                  "fullrl_2x4")
    ev_b = {2: {"bucket": [(0, 0, "in")]}, 30: {"bucket": [(1, 1, "in"), (2, 0, "in")]},
            70: {"bucket": [(0, 1, "in"), (3, 0, "in"), (1, 0, "edge_x")]},
            90: {"force": (3, 4, 350.0)}, 140: {"oob": [(4, "z")]}, 200: {"bucket": [(0, 1, "in")]},
            # two cubes in different buckets in one step: the reference reuses bucket-0 indices for
            # bucket 1 after popping (task_utils.py:103-113) -> pops the wrong cube
            150: {"need": 3, "bucket": [(0, 0, "in"), (1, 1, "in")]},
            230: {"need": 3, "bucket": [(0, 0, "in"), (1, 1, "in")]},
            260: {"oob": [(5, "y")]}}
    meta["fixtures"]["fullrl_4x16"] = gen_episodes("AllFullRLProgressRewardEnv", 4, 16, 42, 320, ev_b, prog,
                                                   "fullrl_4x16", act_seed=3)
    meta["fixtures"]["fullrl_2x8_s7"] = gen_episodes("AllFullRLProgressRewardEnv", 2, 8, 7, 260, ev_a, prog,
                                                     "fullrl_2x8_s7", act_seed=5)
    score_kw = dict(gripper_to_closest_cube_reward_factor=0.0, closest_cube_to_bucket_reward_factor=0.0,
                    small_action_norm_reward_factor=0.0, base_reward=0.0)
    meta["fixtures"]["fullrl_2x10_score"] = gen_episodes("AllFullRLProgressRewardEnv", 2, 10, 42, 200, ev_a,
                                                         score_kw, "fullrl_2x10_score", act_seed=9)
    with open(os.path.join(OUT, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    if "--ik" in sys.argv:
        _setup()
        main_ik()
    else:
        main()
