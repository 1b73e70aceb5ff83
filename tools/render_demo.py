#!/usr/bin/env python3
"""Render a 4x4 grid of arenas (fm_render) after a random-action pre-roll, time the batched render, save a PNG."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--arenas", type=int, default=4096)
ap.add_argument("--preroll", type=int, default=120)
ap.add_argument("--size", type=int, default=240)
ap.add_argument("--out", default="render_demo.png")
a = ap.parse_args()
import torch  # noqa: E402

from factory_marl_amd import FactoryVecEnv  # noqa: E402
from factory_marl_amd.environments import run_kwargs  # noqa: E402

env = FactoryVecEnv(a.arenas, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42),
                    seeds=np.arange(a.arenas))
env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for _ in range(a.preroll):
    env.step_tensors(torch.rand(a.arenas, env.act_dim, device="cuda", generator=g) * 2 - 1)
grid = env.render(indices=range(16), width=a.size, height=a.size)
torch.cuda.synchronize()
for n in (16, 256, a.arenas):
    env.render_tensors(indices=range(n), width=a.size, height=a.size)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(3):
        env.render_tensors(indices=range(n), width=a.size, height=a.size)
    torch.cuda.synchronize()
    dt = (time.time() - t0) / 3
    print(f"render {n} arenas at {a.size}x{a.size}: {dt * 1e3:.2f} ms ({n / dt:.0f} frames/s)")
from PIL import Image  # noqa: E402

Image.fromarray(grid).save(a.out)
print("saved", a.out, grid.shape)
