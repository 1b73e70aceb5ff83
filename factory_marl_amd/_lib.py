"""ctypes binding of libfactorysim.so (the C ABI in include/factorysim.h).

The product path is the HIP library only: if ``libfactorysim.so`` is missing or cannot be loaded this
module raises -- there is no CPU fallback.  ``libfactorysim_exp.so`` is the experiment build of the same sources
(``load(experimental=True)``): its kernels carry the A/B and test switches (FactoryVecEnv.set_experiment) that the
product kernels are compiled without.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FACTORYSIM_LIB", os.path.join(_HERE, "libfactorysim.so"))
EXP_LIB_PATH = os.environ.get("FACTORYSIM_EXP_LIB", os.path.join(_HERE, "libfactorysim_exp.so"))

# env classes (include/factorysim.h FM_ENV_*)
FM_ENV_FACTORY = 0
FM_ENV_ALLFULLRL_PROGRESS = 1
FM_ENV_SINGLEFULLRL_PROGRESS = 2
FM_ENV_SINGLEDELTA_PROGRESS = 3
FM_ENV_ALLDELTA_PROGRESS = 4
FM_ENV_PAUSE_IK_TOGGLE = 5
FM_ENV_BACKUP_IK_TOGGLE = 6
FM_FP32 = 0
FM_FP64 = 1


class FmConfig(C.Structure):
    _fields_ = [
        ("num_arenas", C.c_int32),
        ("num_arms", C.c_int32),
        ("max_num_objects", C.c_int32),
        ("env_class", C.c_int32),
        ("precision", C.c_int32),
        ("max_contacts", C.c_int32),
        ("initial_conveyor_speed", C.c_double),
        ("conveyor_acceleration", C.c_double),
        ("pt_time", C.c_double),
        ("force_contact_threshold", C.c_double),
        ("control_frequency", C.c_double),
        ("spawn_freq", C.c_double),
        ("spawn_freq_increase", C.c_double),
        ("gripper_to_closest_cube_reward_factor", C.c_double),
        ("closest_cube_to_bucket_reward_factor", C.c_double),
        ("small_action_norm_reward_factor", C.c_double),
        ("base_reward", C.c_double),
        ("solver_iterations", C.c_int32),
        ("solver_tolerance", C.c_double),
        ("obs_float64", C.c_int32),
    ]


class FmInfo(C.Structure):
    _fields_ = [
        ("scores", C.c_void_p),
        ("num_obj", C.c_void_p),
        ("play_time", C.c_void_p),
        ("conveyor_speed", C.c_void_p),
        ("out_of_reach", C.c_void_p),
        ("force_terminate", C.c_void_p),
        ("terminal_obs", C.c_void_p),
        ("episode_return", C.c_void_p),
        ("episode_length", C.c_void_p),
        ("terminal_scores", C.c_void_p),
    ]


EXPORTED = [
    "fm_config_default", "fm_create", "fm_destroy", "fm_last_error", "fm_set_stream", "fm_sync", "fm_obs_dim",
    "fm_act_dim", "fm_num_arenas", "fm_nq", "fm_nv", "fm_nu", "fm_workspace_bytes", "fm_reset", "fm_step", "fm_state_size",
    "fm_get_state", "fm_set_state", "fm_get_counters", "fm_debug_dump", "fm_profile", "fm_scene_mjcf",
    "fm_render", "fm_render_ngeom", "fm_set_param", "fm_get_param", "fm_num_counters", "fm_get_costs",
    "fm_kernel_timing", "fm_get_kernel_time", "fm_abi_version", "fm_config_size",
]
ABI_VERSION = 2  # include/factorysim.h FM_ABI_VERSION

_LIBS = {}


class FactorySimError(RuntimeError):
    pass


def load(experimental=False):
    """Load the HIP library (raises if it is missing: the product has no fallback path); experimental: the
    experiment build (libfactorysim_exp.so, A/B and test switches compiled in)."""
    path = EXP_LIB_PATH if experimental else LIB_PATH
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise FactorySimError(f"{path} not built: run `python __graft_entry__.py build` (hipcc, gfx950)")
    L = C.CDLL(path)
    P, I = C.c_void_p, C.c_int
    # the header this binding mirrors (FM_ABI_VERSION, sizeof(fm_config)) must be the library's
    L.fm_abi_version.argtypes = []
    L.fm_abi_version.restype = I
    L.fm_config_size.argtypes = []
    L.fm_config_size.restype = I
    if L.fm_abi_version() != ABI_VERSION or L.fm_config_size() != C.sizeof(FmConfig):
        raise FactorySimError(f"{path}: ABI version {L.fm_abi_version()} / fm_config {L.fm_config_size()} B, this "
                              f"binding expects {ABI_VERSION} / {C.sizeof(FmConfig)} B (rebuild the library)")
    L.fm_config_default.argtypes = [C.POINTER(FmConfig)]
    L.fm_config_default.restype = None
    L.fm_create.argtypes = [C.POINTER(FmConfig), I, C.POINTER(C.c_uint64), C.POINTER(P)]
    L.fm_create.restype = I
    L.fm_destroy.argtypes = [P]
    L.fm_destroy.restype = None
    L.fm_last_error.argtypes = []
    L.fm_last_error.restype = C.c_char_p
    L.fm_set_stream.argtypes = [P, P]
    L.fm_set_stream.restype = I
    L.fm_sync.argtypes = [P]
    L.fm_sync.restype = I
    for n in ["fm_obs_dim", "fm_act_dim", "fm_num_arenas", "fm_nq", "fm_nv", "fm_nu", "fm_workspace_bytes", "fm_state_size"]:
        getattr(L, n).argtypes = [P]
        getattr(L, n).restype = I
    L.fm_reset.argtypes = [P, P, P]
    L.fm_reset.restype = I
    L.fm_step.argtypes = [P, P, P, P, P, P, C.POINTER(FmInfo)]
    L.fm_step.restype = I
    L.fm_get_state.argtypes = [P, P]
    L.fm_get_state.restype = I
    L.fm_set_state.argtypes = [P, P]
    L.fm_set_state.restype = I
    L.fm_get_counters.argtypes = [P, P]
    L.fm_get_counters.restype = I
    L.fm_get_costs.argtypes = [P, P]
    L.fm_get_costs.restype = I
    L.fm_kernel_timing.argtypes = [P, I]
    L.fm_kernel_timing.restype = I
    L.fm_get_kernel_time.argtypes = [P, P, P]
    L.fm_get_kernel_time.restype = I
    L.fm_debug_dump.argtypes = [P, I, I, P, I]
    L.fm_debug_dump.restype = I
    L.fm_profile.argtypes = [P, I, P]
    L.fm_profile.restype = I
    L.fm_scene_mjcf.argtypes = [I, I, C.c_uint64, C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
    L.fm_scene_mjcf.restype = I
    L.fm_render.argtypes = [P, C.POINTER(C.c_int32), I, I, I, C.POINTER(C.c_float), P, P]
    L.fm_render.restype = I
    L.fm_render_ngeom.argtypes = [P]
    L.fm_render_ngeom.restype = I
    L.fm_set_param.argtypes = [P, C.c_char_p, C.c_double]
    L.fm_set_param.restype = I
    L.fm_get_param.argtypes = [P, C.c_char_p, C.POINTER(C.c_double)]
    L.fm_get_param.restype = I
    if hasattr(L, "fm_num_counters"):
        L.fm_num_counters.argtypes = []
        L.fm_num_counters.restype = I
    _LIBS[path] = L
    return L


def num_counters(L):
    """per-arena diagnostic counters of the library (fm_num_counters; libraries before it exported 8)"""
    return L.fm_num_counters() if hasattr(L, "fm_num_counters") else 8


def check(rc, L=None):
    """raise on a nonzero status code with the library's error text (L: the library that returned it)"""
    if rc != 0:
        raise FactorySimError(f"factorysim error {rc}: {(L or load()).fm_last_error().decode()}")


def scene_mjcf(num_arms=2, max_num_objects=10, seed=42, meshdir=None):
    """The compiled scene as an MJCF string (include/factorysim.h fm_scene_mjcf; scene.py:109-161)."""
    L = load()
    n = C.c_size_t(0)
    md = meshdir.encode() if meshdir else None
    check(L.fm_scene_mjcf(num_arms, max_num_objects, seed, md, None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value + 1)
    check(L.fm_scene_mjcf(num_arms, max_num_objects, seed, md, buf, n.value + 1, C.byref(n)))
    return buf.value.decode()
