#!/usr/bin/env python3
"""Which state entries set the teacher-forced fp32 error (test infrastructure, oracle = checker).

For each teacher-forced env-step: the qpos/qvel entry with the largest SURVEY §8(d) relative error, its
reference value and the GPU value; then a histogram of the worst entries over the trajectory.
usage: python tools/worst_dofs.py [--prec fp32] [--traj A,K,T,seed ...]
"""
import argparse
import collections
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import parity_util as pu  # noqa: E402
from parity_sweep import load_traj  # noqa: E402
from oracle import pyoracle as po  # noqa: E402  (checker)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--traj", nargs="*", default=["2,4,96,7", "2,4,300,21"])
    args = ap.parse_args()
    po.build()
    import torch
    from factory_marl_amd import state as st
    for spec in args.traj:
        A, K, T, seed = (int(x) for x in spec.split(","))
        recs, acts, outs = load_traj(A, K, T, seed)
        nq, nv = 1 + 7 * K + 9 * A, 1 + 6 * K + 9 * A
        env = pu.gpu_env(len(recs), args.prec, A, K)
        env.set_state(recs)
        env.step_tensors(torch.as_tensor(acts, device=env.device))
        env.sync()
        got = env.get_state()
        env.close()
        hist = collections.Counter()
        rows = []
        for s in range(len(recs)):
            if outs[s]["term"]:
                continue
            gd, _, _ = st.unpack(A, K, got[s])
            qd, vd = pu.state_err(A, K, gd, outs[s]["dbl"])
            e = np.concatenate([qd, vd])
            j = int(np.argmax(e))
            name = f"qpos[{j}]" if j < nq else f"qvel[{j - nq}]"
            hist[name] += 1
            rows.append(dict(step=s, worst=name, rel=float(e[j]), ref=float(outs[s]["dbl"][j]), got=float(gd[j]),
                             second=float(np.sort(e)[-2]), ncubes=int(outs[s]["info"]["num_obj"])))
        print(json.dumps(dict(traj=spec, prec=args.prec, hist=hist.most_common(12))), flush=True)
        for r in rows[:40]:
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
