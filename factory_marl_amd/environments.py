"""The env classes of src/environments.py as construction specs for the batched GPU path.

``src/learning.py:98-100`` builds its vector env as

    make_vec_env(lambda: Monitor(getattr(environments, CONFIG["env_class"])(**CONFIG["env_kwargs"])),
                 n_envs=CONFIG["num_envs"], vec_env_cls=SubprocVecEnv)

With ``from factory_marl_amd import environments, make_vec_env, Monitor, FactoryVecEnv`` the same line with
``vec_env_cls=FactoryVecEnv`` builds one ``FactoryVecEnv`` of ``num_envs`` arenas: each thunk returns an
``EnvSpec`` (the class name and its fully resolved keyword arguments -- no MuJoCo model is built per env), and
``FactoryVecEnv`` turns the list of specs into one handle.

The constructors accept exactly what the reference's accept and raise ``TypeError`` where it would:
``BaseEnv.__init__`` keywords (base_env.py:15-35) for every class; ``ProgressRewardEnv`` additionally REQUIRES
``gripper_to_closest_cube_reward_factor``, ``closest_cube_to_bucket_reward_factor`` and
``small_action_norm_reward_factor`` and defaults ``base_reward`` to 0.0 (environments.py:252-258); the other classes
reject the reward keywords (their ``**kwargs`` reach ``BaseEnv``, which has no such parameter).
"""
import numpy as np

# BaseEnv.__init__ (base_env.py:15-35)
BASE_DEFAULTS = dict(
    render_mode=None, seed=None, width=480, height=480, camera_id=None, camera_name=None, default_camera_config=None,
    max_geom=1000, visual_options={}, initial_conveyor_speed=0.1, conveyor_acceleration=0.001, pt_time=0.2,
    force_contact_threshold=200.0, max_num_objects=10, control_frequency=10, spawn_freq=1 / 10,
    spawn_freq_increase=1.001, num_arms=2,
)
# rendering-only keywords: accepted, no effect on the batch path (the GPU renderer takes its own camera)
RENDER_ONLY = ("render_mode", "width", "height", "camera_id", "camera_name", "default_camera_config", "max_geom",
               "visual_options")
PROGRESS_REQUIRED = ("gripper_to_closest_cube_reward_factor", "closest_cube_to_bucket_reward_factor",
                     "small_action_norm_reward_factor")
PROGRESS_DEFAULTS = dict(base_reward=0.0)

PROGRESS_CLASSES = ("ProgressRewardEnv", "SingleFullRLProgressRewardEnv", "SingleDeltaProgressRewardEnv",
                    "AllFullRLProgressRewardEnv", "AllDeltaProgressRewardEnv")
TOGGLE_CLASSES = ("PauseIKToggleEnv", "BackupIKToggleEnv")
# the reward weights of the saved progress-reward runs (runs/rk5rxnav.json, runs/r666unuv.json env_kwargs)
RUN_REWARD_KWARGS = dict(gripper_to_closest_cube_reward_factor=0.2, closest_cube_to_bucket_reward_factor=0.4,
                         small_action_norm_reward_factor=0.0, base_reward=0.4)


def run_kwargs(env_class, **kw):
    """env kwargs for `env_class` with the saved runs' reward weights where the class takes them (progress
    classes); `kw` overrides"""
    out = dict(RUN_REWARD_KWARGS) if env_class in PROGRESS_CLASSES else {}
    out.update(kw)
    return out


# classes with a GPU env-step (ProgressRewardEnv and IKTogglingEnv are base classes: the batch path steps their
# concrete subclasses)
GPU_CLASSES = ("FactoryManipulationEnv", "SingleFullRLProgressRewardEnv", "SingleDeltaProgressRewardEnv",
               "AllFullRLProgressRewardEnv", "AllDeltaProgressRewardEnv", "PauseIKToggleEnv", "BackupIKToggleEnv")


def resolve_kwargs(env_class, kwargs, args=()):
    """the complete keyword set of `env_class(*args, **kwargs)` as the reference resolves it; TypeError where the
    reference's constructor raises"""
    kwargs = dict(kwargs)
    progress = env_class in PROGRESS_CLASSES
    if args:
        if env_class != "ProgressRewardEnv":
            raise TypeError(f"{env_class}.__init__() takes 1 positional argument but {len(args) + 1} were given")
        names = PROGRESS_REQUIRED + ("base_reward",)
        if len(args) > len(names):
            raise TypeError(f"ProgressRewardEnv.__init__() takes at most {len(names) + 1} positional arguments")
        for n, v in zip(names, args):
            if n in kwargs:
                raise TypeError(f"ProgressRewardEnv.__init__() got multiple values for argument '{n}'")
            kwargs[n] = v
    out = dict(BASE_DEFAULTS)
    if progress:
        missing = [n for n in PROGRESS_REQUIRED if n not in kwargs]
        if missing:
            raise TypeError(f"{env_class}.__init__() missing {len(missing)} required keyword-only argument(s): "
                            + ", ".join(repr(m) for m in missing))
        out.update(PROGRESS_DEFAULTS)
        for n in PROGRESS_REQUIRED:
            out[n] = kwargs.pop(n)
        if "base_reward" in kwargs:
            out["base_reward"] = kwargs.pop("base_reward")
    for k, v in kwargs.items():
        if k not in BASE_DEFAULTS:
            raise TypeError(f"BaseEnv.__init__() got an unexpected keyword argument '{k}'")
        out[k] = v
    return out


class EnvSpec:
    """one env of the reference, as the batch path needs it: the class name and its resolved keywords"""

    env_class = None

    def __init__(self, *args, **kwargs):
        self.kwargs = resolve_kwargs(self.env_class, kwargs, args)
        A, K = int(self.kwargs["num_arms"]), int(self.kwargs["max_num_objects"])
        self.num_arms, self.max_num_objects = A, K
        self.obs_dim = 24 * A + 13 * K + (8 * A if self.env_class in TOGGLE_CLASSES else 0)
        if self.env_class == "FactoryManipulationEnv":
            self.act_dim = 0
        elif self.env_class in ("SingleFullRLProgressRewardEnv", "SingleDeltaProgressRewardEnv"):
            self.act_dim = 8
        elif self.env_class in TOGGLE_CLASSES:
            self.act_dim = A
        else:
            self.act_dim = 8 * A

    def __eq__(self, other):
        return isinstance(other, EnvSpec) and other.env_class == self.env_class and _same(other.kwargs, self.kwargs)

    def __repr__(self):
        return f"{self.env_class}(**{self.kwargs!r})"


def _same(a, b):
    if a.keys() != b.keys():
        return False
    return all(np.array_equal(np.asarray(a[k], dtype=object), np.asarray(b[k], dtype=object)) for k in a)


def _spec_class(name):
    return type(name, (EnvSpec,), {"env_class": name, "__doc__": f"{name} (src/environments.py) as an EnvSpec"})


FactoryManipulationEnv = _spec_class("FactoryManipulationEnv")
ProgressRewardEnv = _spec_class("ProgressRewardEnv")
SingleFullRLProgressRewardEnv = _spec_class("SingleFullRLProgressRewardEnv")
SingleDeltaProgressRewardEnv = _spec_class("SingleDeltaProgressRewardEnv")
AllFullRLProgressRewardEnv = _spec_class("AllFullRLProgressRewardEnv")
AllDeltaProgressRewardEnv = _spec_class("AllDeltaProgressRewardEnv")
IKTogglingEnv = _spec_class("IKTogglingEnv")
PauseIKToggleEnv = _spec_class("PauseIKToggleEnv")
BackupIKToggleEnv = _spec_class("BackupIKToggleEnv")


def Monitor(env, filename=None, allow_early_resets=True, reset_keywords=(), info_keywords=(), override_existing=True):
    """stable_baselines3.common.monitor.Monitor stand-in: the batch env records the Monitor episode statistics itself
    (infos[i]["episode"] = {"r", "l", "t"}), so the wrapper passes the spec through.  CSV logging (filename) is not
    provided."""
    if filename is not None:
        raise NotImplementedError("Monitor CSV files are not written by the batch path (infos carry the episodes)")
    return env
