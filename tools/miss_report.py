#!/usr/bin/env python3
"""Teacher-forced fp32 misses in detail (test infrastructure): for every env-step over the SURVEY gate, the worst
state entry (body / dof, reference value, GPU value) and the step's contact context.
usage: FACTORYSIM_LIB=... FM_TRAJ_CACHE=traj_cache python tools/miss_report.py [--prec fp32] [--traj A,K,T,seed ...]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import parity_util as pu  # noqa: E402
import parity_sweep as ps  # noqa: E402


def dof_name(A, K, j, nq):
    if j < nq:
        if j == 0:
            return "qpos belt"
        if j < 1 + 7 * K:
            return f"qpos cube{(j - 1) // 7}[{(j - 1) % 7}]"
        return f"qpos arm{(j - 1 - 7 * K) // 9}[{(j - 1 - 7 * K) % 9}]"
    j -= nq
    if j == 0:
        return "qvel belt"
    if j < 1 + 6 * K:
        return f"qvel cube{(j - 1) // 6}[{(j - 1) % 6}]"
    return f"qvel arm{(j - 1 - 6 * K) // 9}[{(j - 1 - 6 * K) % 9}]"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--tag", default="")
    ap.add_argument("--traj", nargs="*", default=["2,4,96,7", "2,4,300,21", "2,8,300,5", "2,10,250,9"])
    args = ap.parse_args()
    for spec in args.traj:
        A, K, T, seed = (int(x) for x in spec.split(","))
        recs, acts, outs = ps.load_traj(A, K, T, seed)
        r = pu.compare((recs, acts, outs), args.prec, A, K)
        import torch  # noqa: F401
        nq = 1 + 7 * K + 9 * A
        env = pu.gpu_env(len(recs), args.prec, A, K)
        env.set_state(recs)
        env.step_tensors(torch.as_tensor(acts, device=env.device))
        env.sync()
        got = env.get_state()
        env.close()
        from factory_marl_amd import state as st
        rows = []
        for s in r["err_steps"][r["errs"] > 1e-4]:
            gd, _, _ = st.unpack(A, K, got[s])
            qd, vd = pu.state_err(A, K, gd, outs[s]["dbl"])
            e = np.concatenate([qd, vd])
            top = np.argsort(e)[::-1][:3]
            rows.append(dict(step=int(s), err=float(e.max()), ncubes=int(outs[s]["info"]["num_obj"]),
                             worst=[dict(what=dof_name(A, K, int(j), nq), rel=float(e[j]), ref=float(outs[s]["dbl"][j]),
                                         got=float(gd[j])) for j in top]))
        print(json.dumps(dict(tag=args.tag, traj=spec, within=float(np.mean(r["errs"] <= 1e-4)), misses=rows)), flush=True)


if __name__ == "__main__":
    main()
