"""Bit-identity and timing of the arrowhead Cholesky fast path (chol_arrow_rl) against the general register
Cholesky (FM_NO_ARROW=1) on the (2,4) scene: the same states stepped with the same actions under each switch,
full state records compared bitwise.  The arrowhead factor of the LDS-assembled Hessian (FM_NO_ARROW=2) is
bit-identical to the general one; the default (Hessian assembled in registers) sums in another order.  usage: python tools/arrow_probe.py [--arenas N] [--steps K]"""
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


def run(env, s0, acts, mode):
    """mode "" = default (Hessian assembled in the arrowhead factor's registers), "1" = general register Cholesky,
    "2" = arrowhead factor of the LDS-assembled Hessian"""
    env.set_experiment(f"FM_NO_ARROW={mode}" if mode else "")
    env.set_state(s0)
    env.sync()
    t0 = time.perf_counter()
    for a in acts:
        env.step_tensors(a)
    env.sync()
    dt = time.perf_counter() - t0
    return env.get_state(), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arenas", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--preroll", type=int, default=100)
    args = ap.parse_args()
    out = {}
    for prec in ("fp32", "fp64"):
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
        run(env, s0, acts[:3], "")  # warm
        sa, ta = run(env, s0, acts, "")
        sg, tg = run(env, s0, acts, "1")
        sl, tl = run(env, s0, acts, "2")
        sa2, ta2 = run(env, s0, acts, "")
        out[prec] = dict(arenas=n, steps=args.steps,
                         lds_arrow_vs_general_differing=int((sl != sg).any(axis=1).sum()),
                         reg_asm_vs_general_differing=int((sa != sg).any(axis=1).sum()),
                         rerun_differing=int((sa != sa2).any(axis=1).sum()),
                         ms_per_step_reg_asm=1e3 * min(ta, ta2) / args.steps, ms_per_step_lds_arrow=1e3 * tl / args.steps,
                         ms_per_step_general=1e3 * tg / args.steps)
        print(prec, out[prec], flush=True)
        env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
