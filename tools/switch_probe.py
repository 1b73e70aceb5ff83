"""A/B of the kernel's experiment switches (FactoryVecEnv.set_experiment on the live handle) on the
(2,4) scene: the same states stepped with the same actions under each switch setting; reports per setting the
arenas whose full state record differs bitwise from the first setting's, and the time per env-step.
usage: python tools/switch_probe.py [--arenas N] [--steps K] -- "" FM_NO_SCATTER=1 "FM_NO_ARROW=1 FM_NO_SCATTER=1"
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from factory_marl_amd import FactoryVecEnv  # noqa: E402
from factory_marl_amd.environments import run_kwargs  # noqa: E402

def run(env, s0, acts, setting):
    env.set_experiment(setting)
    env.set_state(s0)
    env.sync()
    t0 = time.perf_counter()
    for a in acts:
        env.step_tensors(a)
    env.sync()
    return env.get_state(), time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arenas", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--preroll", type=int, default=100)
    ap.add_argument("--precisions", default="fp32,fp64")
    ap.add_argument("settings", nargs="+")
    args = ap.parse_args()
    out = {}
    for prec in args.precisions.split(","):
        n = args.arenas
        env = FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42),
                            precision=prec, seeds=42 + np.arange(n), return_numpy=False, experimental=True)
        env.reset()
        g = torch.Generator(device=env.device)
        g.manual_seed(3)
        for _ in range(args.preroll):
            env.step_tensors(torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1)
        env.sync()
        s0 = env.get_state()
        acts = [torch.rand(n, env.act_dim, device=env.device, generator=g) * 2 - 1 for _ in range(args.steps)]
        run(env, s0, acts[:3], args.settings[0])  # warm
        ref = None
        res = {}
        for s in args.settings:
            st, dt = run(env, s0, acts, s)
            st2, dt2 = run(env, s0, acts, s)
            if ref is None:
                ref = st
            res[s or "default"] = dict(differing_from_first=int((st != ref).any(axis=1).sum()),
                                       rerun_differing=int((st != st2).any(axis=1).sum()),
                                       ms_per_step=1e3 * min(dt, dt2) / args.steps)
        out[prec] = res
        print(prec, json.dumps(res), flush=True)
        env.close()
    apply("")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
