"""ctypes front-end of the oracle (TEST INFRASTRUCTURE ONLY).

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the product
package factory_marl_amd/.  See oracle/oracle.h for what the C library restates.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_LIB_F32 = None


def build(force=False):
    so = os.path.join(_HERE, "liboracle.so")
    srcs = [os.path.join(_HERE, f) for f in os.listdir(_HERE) if f.endswith((".c", ".h"))]
    if force or not os.path.exists(so) or max(os.path.getmtime(s) for s in srcs) > os.path.getmtime(so):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return so


def lib(f32=False):
    """the oracle library; f32=True loads liboracle_f32.so, the same sources with every double a float (the fp32
    floor study of tools/fp32_floor.py --float-oracle), whose real-valued arguments are float32"""
    global _LIB, _LIB_F32
    if f32:
        if _LIB_F32 is None:
            so = os.path.join(_HERE, "liboracle_f32.so")
            subprocess.run(["make", "-s", "-C", _HERE, "liboracle_f32.so"], check=True)
            _LIB_F32 = _bind(C.CDLL(so), C.c_float)
        return _LIB_F32
    if _LIB is None:
        so = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(so):
            build()
        _LIB = _bind(C.CDLL(so), C.c_double)
    return _LIB


def _bind(L, real):
    if True:
        P, I, D, U64 = C.c_void_p, C.c_int, real, C.c_uint64
        DP = C.POINTER(real)
        sig = {
            "or_env_create": (P, [I, I, U64, I, DP]),
            "or_env_free": (None, [P]), "or_env_set_timing": (None, [P, D, D]),
            "or_env_reset": (None, [P, P]),
            "or_env_step": (I, [P, P, P, DP, DP]),
            "or_env_model": (P, [P]), "or_env_data": (P, [P]), "or_env_task": (P, [P]),
            "or_env_obs_dim": (I, [P]),
            "or_model_create": (P, [I, I, U64]), "or_model_free": (None, [P]),
            "or_data_create": (P, [P]), "or_data_free": (None, [P]),
            "or_m_int": (I, [P, C.c_char_p]), "or_m_meaninertia": (D, [P]),
            "or_m_body_invweight0": (DP, [P]), "or_m_dof_invweight0": (DP, [P]), "or_m_cube_size": (DP, [P]),
            "or_m_body_mass": (DP, [P]), "or_m_geom_body": (C.POINTER(I), [P]),
            "or_m_geom_type": (C.POINTER(I), [P]), "or_m_geom_size": (DP, [P]),
            "or_m_arm_geom_lo": (C.POINTER(I), [P]), "or_m_arm_geom_hi": (C.POINTER(I), [P]),
            "or_m_act_ctrlrange": (DP, [P]), "or_m_grip_site": (I, [P, I]),
            "or_d_qpos": (DP, [P]), "or_d_qvel": (DP, [P]), "or_d_ctrl": (DP, [P]), "or_d_qacc": (DP, [P]),
            "or_d_qacc_warmstart": (DP, [P]), "or_d_M": (DP, [P]), "or_d_qfrc_bias": (DP, [P]),
            "or_d_qfrc_constraint": (DP, [P]), "or_d_xpos": (DP, [P]), "or_d_xmat": (DP, [P]),
            "or_d_xipos": (DP, [P]), "or_d_geom_xpos": (DP, [P]), "or_d_geom_xmat": (DP, [P]),
            "or_d_site_xpos": (DP, [P]), "or_d_efc_force": (DP, [P]),
            "or_d_ncon": (I, [P]), "or_d_nefc": (I, [P]), "or_d_niter": (I, [P]),
            "or_d_set_actuation_disabled": (None, [P, I]),
            "or_d_contact": (None, [P, I, P, P]),
            "or_physics_step": (None, [P, P, P]),
            "or_kinematics": (None, [P, P]), "or_mass": (None, [P, P]), "or_bias": (None, [P, P]),
            "or_step1": (None, [P, P]), "or_step2": (None, [P, P]), "or_forward": (None, [P, P]),
            "or_reset_data": (None, [P, P]),
            "or_jac_point": (None, [P, P, I, P, P, P]),
            "or_contact_force": (None, [P, P, I, P]),
            "or_impedance": (D, [P, D]),
            "or_box_box": (I, [P, P, P, P, P, P, D, P]),
            "or_sphere_box": (I, [P, D, P, P, P, D, P]),
            "or_plane_box": (I, [P, P, P, P, P, D, P]),
            "or_pcg64_seed": (None, [P, U64]), "or_pcg64_next64": (U64, [P]), "or_pcg64_double": (D, [P]),
            "or_task_new": (P, [I, I, U64]), "or_task_free": (None, [P]),
            "or_task_reset": (None, [P, P, P, P]),
            "or_task_process_action": (None, [P, P, P]),
            "or_task_clip_ctrl": (None, [P, P, P, P]),
            "or_task_lowpass": (None, [P, P, P, I, P]),
            "or_task_force_check": (I, [P, P, I, P, P]),
            "or_task_step": (None, [P, P, P, P]),
            "or_task_after_step": (None, [P]),
            "or_task_obs": (None, [P, P, P, P, P]),
            "or_task_reward": (D, [P, P, P, P, P]),
            "or_t_int": (I, [P, C.c_char_p]), "or_t_double": (D, [P, C.c_char_p]),
            "or_t_in_scene": (C.POINTER(I), [P]), "or_t_ctrl_target": (DP, [P]),
            "or_t_set_reward": (None, [P, I, DP]),
            "or_env_export": (None, [P, P, P, P]),
            "or_d_qacc_smooth": (DP, [P]), "or_d_qfrc_smooth": (DP, [P]), "or_d_qfrc_passive": (DP, [P]),
            "or_d_efc_type": (C.POINTER(I), [P]), "or_d_efc_pos": (DP, [P]), "or_d_efc_D": (DP, [P]),
            "or_d_efc_aref": (DP, [P]), "or_d_efc_J": (DP, [P]), "or_d_stage_fwd": (DP, [P, P, I]),
            "or_env_import": (None, [P, P, P, P]),
            "or_batch_bench": (D, [I, I, I, I, I, U64, P]),
            "or_set_accel_noise": (None, [D, U64]), "or_set_solver_tol": (None, [D]),
            "or_set_probe": (None, [I, D, U64]),
            "or_ik_arm_init_flat": (None, [P, P]), "or_ik_arm_reset_flat": (None, [P, P]),
            "or_ik_plan_flat": (I, [I, I, P, P, P, P, P, P, P, P, P, P, P, P]),
            "or_ik_finish_flat": (None, [P, P, I, P, I, P]),
            "or_ik_grasp_quat": (None, [P, P]),
            "or_ik_compose_replay": (I, [P, P, P, P, P, P, P, P, I, P, P, I, P, P]),
            "or_compose_class": (None, [P, I, P, P, P, P, P, P]),
            "or_t_set_ignore": (None, [P, I, P, I]), "or_t_set_in_scene": (None, [P, P, I]),
            "or_t_set_scores": (None, [P, I, I]), "or_t_reset_reward_state": (None, [P]), "or_t_set_act_dim": (None, [P, I]),
            "or_env_act_dim": (I, [P]), "or_env_ik_steps": (I, [P]),
            "or_env_ik_calls": (C.c_long, [P, I]), "or_env_ik_fails": (C.c_long, [P, I]), "or_env_ik_arm": (None, [P, I, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
    L.real = np.float32 if real is C.c_float else np.float64
    L.c_real = real
    return L


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def arr(p, n, dtype=np.float64):
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dtype, copy=True)


# contact record layout of or_contact (oracle.h): 4+9... doubles then 4 ints
CONTACT_BYTES = 8 * (1 + 3 + 9 + 1 + 2 + 5 + 1) + 4 * 4


class Model:
    def __init__(self, A, K, seed, handle=None, L=None):
        L = self.L = L or lib()
        self.own = handle is None
        self.h = handle if handle is not None else L.or_model_create(A, K, seed)
        if not self.h:
            raise ValueError("bad model config")
        for k in ["A", "K", "nbody", "njnt", "nq", "nv", "ngeom", "nsite", "nu", "neq", "cube_body0"]:
            setattr(self, k, L.or_m_int(self.h, k.encode()))

    def __del__(self):
        if getattr(self, "own", False) and self.h:
            self.L.or_model_free(self.h)

    @property
    def cube_size(self):
        return arr(self.L.or_m_cube_size(self.h), self.K)

    @property
    def body_invweight0(self):
        return arr(self.L.or_m_body_invweight0(self.h), 2 * self.nbody).reshape(-1, 2)

    @property
    def dof_invweight0(self):
        return arr(self.L.or_m_dof_invweight0(self.h), self.nv)

    @property
    def meaninertia(self):
        return self.L.or_m_meaninertia(self.h)

    @property
    def ctrlrange(self):
        return arr(self.L.or_m_act_ctrlrange(self.h), 2 * self.nu).reshape(-1, 2)

    @property
    def geom_body(self):
        return arr(self.L.or_m_geom_body(self.h), self.ngeom, np.int32)

    @property
    def geom_type(self):
        return arr(self.L.or_m_geom_type(self.h), self.ngeom, np.int32)

    @property
    def geom_size(self):
        return arr(self.L.or_m_geom_size(self.h), 3 * self.ngeom).reshape(-1, 3)

    @property
    def body_mass(self):
        return arr(self.L.or_m_body_mass(self.h), self.nbody)

    def arm_geom_range(self, i):
        L = self.L
        return L.or_m_arm_geom_lo(self.h)[i], L.or_m_arm_geom_hi(self.h)[i]


class Data:
    def __init__(self, model, handle=None):
        L = self.L = model.L
        self.m = model
        self.own = handle is None
        self.h = handle if handle is not None else L.or_data_create(model.h)

    def __del__(self):
        if getattr(self, "own", False) and self.h:
            self.L.or_data_free(self.h)

    def _view(self, fn, n):
        return np.ctypeslib.as_array(getattr(self.L, fn)(self.h), shape=(n,))

    @property
    def qpos(self):
        return self._view("or_d_qpos", self.m.nq)

    @property
    def qvel(self):
        return self._view("or_d_qvel", self.m.nv)

    @property
    def ctrl(self):
        return self._view("or_d_ctrl", self.m.nu)

    @property
    def qacc(self):
        return self._view("or_d_qacc", self.m.nv)

    @property
    def qacc_warmstart(self):
        return self._view("or_d_qacc_warmstart", self.m.nv)

    @property
    def M(self):
        return self._view("or_d_M", self.m.nv * self.m.nv).reshape(self.m.nv, self.m.nv)

    @property
    def qfrc_bias(self):
        return self._view("or_d_qfrc_bias", self.m.nv)

    @property
    def qfrc_constraint(self):
        return self._view("or_d_qfrc_constraint", self.m.nv)

    @property
    def xpos(self):
        return self._view("or_d_xpos", 3 * self.m.nbody).reshape(-1, 3)

    @property
    def xmat(self):
        return self._view("or_d_xmat", 9 * self.m.nbody).reshape(-1, 3, 3)

    @property
    def xipos(self):
        return self._view("or_d_xipos", 3 * self.m.nbody).reshape(-1, 3)

    @property
    def geom_xpos(self):
        return self._view("or_d_geom_xpos", 3 * self.m.ngeom).reshape(-1, 3)

    @property
    def geom_xmat(self):
        return self._view("or_d_geom_xmat", 9 * self.m.ngeom).reshape(-1, 3, 3)

    @property
    def site_xpos(self):
        return self._view("or_d_site_xpos", 3 * self.m.nsite).reshape(-1, 3)

    @property
    def ncon(self):
        return self.L.or_d_ncon(self.h)

    @property
    def nefc(self):
        return self.L.or_d_nefc(self.h)

    @property
    def niter(self):
        return self.L.or_d_niter(self.h)

    def contacts(self):
        out = []
        g = np.zeros(2, np.int32)
        v = np.zeros(14)
        for i in range(self.ncon):
            self.L.or_d_contact(self.h, i, ptr(g), ptr(v))
            out.append(dict(geom=tuple(int(x) for x in g), dist=v[0], pos=v[1:4].copy(),
                            frame=v[4:13].reshape(3, 3).copy(), mu=v[13]))
        return out

    def contact_force(self, i):
        f = np.zeros(6)
        self.L.or_contact_force(self.m.h, self.h, i, ptr(f))
        return f

    def step(self, ctrl=None):
        c = np.zeros(self.m.nu, self.L.real) if ctrl is None else np.ascontiguousarray(ctrl, dtype=self.L.real)
        self.L.or_physics_step(self.m.h, self.h, ptr(c))

    def forward(self):
        self.L.or_forward(self.m.h, self.h)

    def step1(self):
        self.L.or_step1(self.m.h, self.h)

    def jac(self, body, point):
        p = np.ascontiguousarray(point, dtype=np.float64)
        jp = np.zeros(3 * self.m.nv)
        jr = np.zeros(3 * self.m.nv)
        self.L.or_jac_point(self.m.h, self.h, body, ptr(p), ptr(jp), ptr(jr))
        return jp.reshape(3, -1), jr.reshape(3, -1)


# env classes of src/environments.py (oracle.h OR_ENV_*, include/factorysim.h FM_ENV_*)
ENV_CLASSES = {"FactoryManipulationEnv": 0, "AllFullRLProgressRewardEnv": 1, "SingleFullRLProgressRewardEnv": 2,
               "SingleDeltaProgressRewardEnv": 3, "AllDeltaProgressRewardEnv": 4, "PauseIKToggleEnv": 5,
               "BackupIKToggleEnv": 6}
IK_STATES = ["IDLE", "GO_TO_GRASP", "GRASP_APPROACH", "GRASP_CLOSE", "POST_GRASP", "GO_TO_RELEASE", "RELEASE"]


class Env:
    """Oracle restatement of the env classes of src/environments.py (default AllFullRLProgressRewardEnv)."""

    def __init__(self, num_arms=2, max_num_objects=4, seed=42, reward="progress",
                 weights=(0.2, 0.4, 0.0, 0.4), env_class=None, f32=False, pt_time=0.2, control_frequency=10):
        L = self.L = lib(f32)
        w = (L.c_real * 4)(*weights)
        if env_class is None:  # legacy selector: progress -> AllFullRL, score -> FactoryManipulationEnv
            env_class = "AllFullRLProgressRewardEnv" if reward == "progress" else "FactoryManipulationEnv"
        self.env_class = env_class
        self.h = L.or_env_create(num_arms, max_num_objects, seed, ENV_CLASSES[env_class], w)
        if not self.h:
            raise ValueError("bad env config")
        if (pt_time, control_frequency) != (0.2, 10):
            L.or_env_set_timing(self.h, pt_time, control_frequency)
        self.model = Model(num_arms, max_num_objects, seed, handle=L.or_env_model(self.h), L=L)
        self.data = Data(self.model, handle=L.or_env_data(self.h))
        self.task = L.or_env_task(self.h)
        self.obs_dim = L.or_env_obs_dim(self.h)
        self.act_dim = L.or_env_act_dim(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.or_env_free(self.h)
            self.h = None

    def reset(self):
        obs = np.zeros(self.obs_dim, np.float32)
        self.L.or_env_reset(self.h, ptr(obs))
        return obs

    def step(self, action):
        a = np.ascontiguousarray(action if self.act_dim else np.zeros(1), dtype=np.float32)
        obs = np.zeros(self.obs_dim, np.float32)
        rew = self.L.c_real(0)
        info = (self.L.c_real * 7)()
        term = self.L.or_env_step(self.h, ptr(a), ptr(obs), C.byref(rew), info)
        inf = dict(scores=[int(info[0]), int(info[1])], play_time=info[2], conveyor_speed=info[3],
                   out_of_reach=bool(info[4]), force_terminate=bool(info[5]), num_obj=int(info[6]))
        return obs, rew.value, bool(term), False, inf

    def task_int(self, what):
        return self.L.or_t_int(self.task, what.encode())

    def task_double(self, what):
        return self.L.or_t_double(self.task, what.encode())

    def in_scene(self):
        n = self.task_int("n_in")
        p = self.L.or_t_in_scene(self.task)
        return [p[i] for i in range(n)]

    def ctrl_target(self):
        return arr(self.L.or_t_ctrl_target(self.task), self.model.nu)

    def state_sizes(self):
        m = self.model
        nd = 2 * m.nq + 3 * m.nv + m.nu + 3 + 2 * m.A + 1 + 27 * m.A
        ni = 2 * m.K + 11 + (3 + m.A) * m.A
        return nd, ni

    def ik_arm(self, i):
        """IKPolicy state of arm i: dict(state, counter, target, ignore, last_ctrl, move_start)"""
        ai = np.zeros(19, np.int32)
        ad = np.zeros(11)
        self.L.or_env_ik_arm(self.h, i, ptr(ai), ptr(ad))
        return dict(state=int(ai[0]), counter=int(ai[1]), target=int(ai[2]), ignore=list(ai[3:3 + self.model.A]),
                    last_ctrl=ad[:8].copy(), move_start=ad[8:11].copy())

    def ik_steps(self):
        return self.L.or_env_ik_steps(self.h)

    def ik_solve_counts(self, arm):
        """(IK solves, failed solves) of arm `arm` since creation (diagnostics)"""
        return int(self.L.or_env_ik_calls(self.h, arm)), int(self.L.or_env_ik_fails(self.h, arm))

    def export_state(self):
        """full arena state in the product's record layout (fm_get_state)"""
        nd, ni = self.state_sizes()
        dbl = np.zeros(nd, self.L.real)
        ints = np.zeros(ni, np.int32)
        rng = np.zeros(4, np.uint64)
        self.L.or_env_export(self.h, ptr(dbl), ptr(ints), ptr(rng))
        return dbl, ints, rng

    def import_state(self, dbl, ints, rng):
        dbl = np.ascontiguousarray(dbl, dtype=self.L.real)
        ints = np.ascontiguousarray(ints, dtype=np.int32)
        rng = np.ascontiguousarray(rng, dtype=np.uint64)
        self.L.or_env_import(self.h, ptr(dbl), ptr(ints), ptr(rng))
