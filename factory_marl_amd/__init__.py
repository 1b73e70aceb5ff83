"""factory_marl_amd -- MI355X-native batched env-step path of nkirschi/Factory-MARL.

The reference steps one MuJoCo arena per Python process (challenge_env BaseEnv.step_sim +
src/environments.py wrappers, driven by SB3 SubprocVecEnv).  Here every arena lives in HBM and one
hand-written HIP kernel (csrc/fm_device.hpp, instantiated by csrc/fm_api.hip and csrc/fm_fixed.hip) advances all of them per env-step; FactoryVecEnv exposes
the SB3 VecEnv surface over it.  See DESIGN.md.
"""
from . import environments  # noqa: F401
from ._lib import FactorySimError, load  # noqa: F401
from .environments import Monitor  # noqa: F401
from .vec_env import FactoryVecEnv, make_vec_env  # noqa: F401

__all__ = ["FactoryVecEnv", "FactorySimError", "load", "environments", "make_vec_env", "Monitor"]
