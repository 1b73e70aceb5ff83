#!/usr/bin/env python3
"""GPU parity sweep (test infrastructure): teacher-forced trajectories through one library build / precision /
solver setting, one JSON line per trajectory (tests/parity_util.summary + the setting).

usage: FACTORYSIM_LIB=path python tools/parity_sweep.py --prec fp32 [--tol 1e-9] [--tag name]
           [--traj A,K,T,seed[,EnvClass[,oracle_tol]] ...]   (default: 2,4,96,7  2,4,300,21  2,8,300,5  2,10,250,9)
Trajectories are cached as .npz under gpurun_out/traj/ (or $FM_TRAJ_CACHE: a cache made in the container travels
with the tree) so several processes share one oracle rollout.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import parity_util as pu  # noqa: E402
from oracle import pyoracle as po  # noqa: E402  (checker)


def load_traj(A, K, T, seed, env_class="AllFullRLProgressRewardEnv",
              cache=os.environ.get("FM_TRAJ_CACHE", os.path.join(ROOT, "gpurun_out", "traj")), oracle_tol=0.0):
    """oracle_tol > 0: the expected outputs come from an oracle whose Newton stops at that tolerance (MuJoCo's
    default 1e-8), stepped from the same states (tools/tolerance_floor.py --make-traj writes those files)"""
    os.makedirs(cache, exist_ok=True)
    tag = "" if env_class == "AllFullRLProgressRewardEnv" else "_" + env_class
    if oracle_tol > 0:
        tag += f"_tol{oracle_tol:g}"
    f = os.path.join(cache, f"traj_{A}_{K}_{T}_{seed}{tag}.npz")
    if oracle_tol > 0 and not os.path.exists(f):
        raise FileNotFoundError(f + " (make it with tools/tolerance_floor.py --make-traj)")
    if os.path.exists(f):
        z = np.load(f)
        meta = json.load(open(f[:-4] + ".json"))
        outs = []
        for s in range(T):
            outs.append(dict(obs=z["obs"][s], reward=float(z["reward"][s]), term=bool(z["term"][s]),
                             info=meta["info"][s], dbl=z["dbl"][s], ints=z["ints"][s], rng=z["rng"][s]))
        return z["recs"], z["acts"], outs
    recs, acts, outs = pu.rollout(po, A, K, T, seed_actions=seed, env_class=env_class)
    np.savez(f, recs=recs, acts=acts, obs=np.stack([o["obs"] for o in outs]),
             reward=np.array([o["reward"] for o in outs]), term=np.array([o["term"] for o in outs]),
             dbl=np.stack([o["dbl"] for o in outs]), ints=np.stack([o["ints"] for o in outs]),
             rng=np.stack([o["rng"] for o in outs]))
    json.dump(dict(info=[o["info"] for o in outs]), open(f[:-4] + ".json", "w"))
    return recs, acts, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--tol", type=float, default=0.0)
    ap.add_argument("--iters", type=int, default=0)
    ap.add_argument("--tag", default="")
    ap.add_argument("--traj", nargs="*", default=["2,4,96,7", "2,4,300,21", "2,8,300,5", "2,10,250,9"])
    args = ap.parse_args()
    po.build()
    for spec in args.traj:
        f = spec.split(",")
        A, K, T, seed = (int(x) for x in f[:4])
        env_class = f[4] if len(f) > 4 and f[4] else "AllFullRLProgressRewardEnv"
        otol = float(f[5]) if len(f) > 5 else 0.0
        t0 = time.time()
        traj = load_traj(A, K, T, seed, env_class, oracle_tol=otol)
        t1 = time.time()
        r = pu.compare(traj, args.prec, A, K, env_class, solver_tolerance=args.tol, solver_iterations=args.iters)
        s = pu.summary(r)
        s.update(tag=args.tag, lib=os.path.basename(os.environ.get("FACTORYSIM_LIB", "libfactorysim.so")),
                 prec=args.prec, tol=args.tol,
                 traj=spec, rollout_s=round(t1 - t0, 1), gpu_s=round(time.time() - t1, 1))
        print(json.dumps(s), flush=True)


if __name__ == "__main__":
    main()
