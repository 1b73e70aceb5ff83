import os, sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from factory_marl_amd import FactoryVecEnv
from factory_marl_amd.environments import run_kwargs
for prec in ("fp64", "fp32"):
    n = 256
    env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42), precision=prec, seeds=42 + np.arange(n), return_numpy=False)
    env.reset(); s0 = env.get_state()
    g = torch.Generator(device=env.device); g.manual_seed(5)
    acts = [torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1 for _ in range(40)]
    outs = []
    for rep in range(3):
        env.set_state(s0)
        for k, a in enumerate(acts):
            env.step_tensors(a)
        env.sync(); outs.append(env.get_state())
    d = [int((outs[0] != o).any(axis=1).sum()) for o in outs[1:]]
    print(prec, "arenas differing from run 0:", d, flush=True)
    env.close()
