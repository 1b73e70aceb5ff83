#!/usr/bin/env python3
"""Dump the obs / state after 30 random env-steps of 4096 (2,4) arenas from the library FACTORYSIM_LIB names
(variant builds of tools/build_variant.sh), so two builds can be compared bit for bit.  usage: variant_obs.py OUT.npy"""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from factory_marl_amd import FactoryVecEnv  # noqa: E402
from factory_marl_amd.environments import run_kwargs  # noqa: E402

env = FactoryVecEnv(4096, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42), precision="fp32")
env.reset()
g = torch.Generator(device=env.device)
g.manual_seed(0)
for _ in range(30):
    env.step_tensors(torch.rand(4096, 16, device=env.device, generator=g) * 2 - 1)
env.sync()
np.save(sys.argv[1], np.concatenate([env.obs.cpu().numpy().ravel().view(np.uint8), np.ascontiguousarray(env.get_state()).ravel().view(np.uint8)]))
env.close()
