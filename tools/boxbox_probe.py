"""fp64: first env-step at which the wave-parallel and the serial box-box narrowphase diverge (test infrastructure)"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import parity_util as pu
from factory_marl_amd import FactoryVecEnv
from factory_marl_amd import state as st
from factory_marl_amd.environments import run_kwargs
n = 256
env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42), precision="fp64", seeds=42 + np.arange(n), return_numpy=False)
env.reset(); s0 = env.get_state()
g = torch.Generator(device=env.device); g.manual_seed(5)
acts = [torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1 for _ in range(40)]
traj = []
for on in (False, True):
    env.set_state(s0)
    if on: os.environ["FM_SERIAL_BOXBOX"] = "1"
    states = []
    for a in acts:
        env.step_tensors(a); env.sync(); states.append(env.get_state())
    os.environ.pop("FM_SERIAL_BOXBOX", None)
    traj.append(states)
for k in range(40):
    a, b = traj[0][k], traj[1][k]
    diff = np.nonzero((a != b).any(axis=1))[0]
    if len(diff):
        w = max(max(m.max() for m in pu.state_err(2, 4, st.unpack(2, 4, a[i])[0], st.unpack(2, 4, b[i])[0])) for i in diff)
        print(f"step {k}: {len(diff)} arenas differ, worst relative {w:.2e}", flush=True)
print("done")
