#!/usr/bin/env python3
"""GPU parity sweep (test infrastructure): teacher-forced trajectories through one library build / precision /
solver setting, one JSON line per trajectory (tests/parity_util.summary + the setting).

usage: FACTORYSIM_LIB=path python tools/parity_sweep.py --prec fp32 [--tol 1e-9] [--tag name]
           [--traj A,K,T,seed[,EnvClass[,oracle_tol]] ...]   (default: 2,4,96,7  2,4,300,21  2,8,300,5  2,10,250,9)
       python tools/parity_sweep.py --make-only --workers 8 --traj ...   (oracle rollouts into the cache, no GPU)
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
        # the tight oracle's states and actions, restepped at the given Newton tolerance
        trj = pu.restep_at_tolerance(po, A, K, load_traj(A, K, T, seed, env_class, cache), oracle_tol, env_class)
        _save(f, *trj)
    if os.path.exists(f):
        z = np.load(f)
        meta = json.load(open(f[:-4] + ".json"))
        outs = []
        for s in range(T):
            outs.append(dict(obs=z["obs"][s], reward=float(z["reward"][s]), term=bool(z["term"][s]),
                             info=meta["info"][s], dbl=z["dbl"][s], ints=z["ints"][s], rng=z["rng"][s]))
            if outs[-1]["term"] and "reset_dbl" in z:
                outs[-1]["reset"] = {k: z["reset_" + k][s] for k in ("obs", "dbl", "ints", "rng")}
        return z["recs"], z["acts"], outs
    recs, acts, outs = pu.rollout(po, A, K, T, seed_actions=seed, env_class=env_class)
    _save(f, recs, acts, outs)
    return recs, acts, outs


def _save(f, recs, acts, outs):
    extra = {}
    rs = [o.get("reset") for o in outs]
    if any(r is not None for r in rs):
        # the oracle's post-auto-reset record of terminating steps (zeros elsewhere)
        r0 = next(r for r in rs if r is not None)
        for k in ("obs", "dbl", "ints", "rng"):
            extra["reset_" + k] = np.stack([r[k] if r is not None else np.zeros_like(r0[k]) for r in rs])
    np.savez(f, recs=recs, acts=acts, obs=np.stack([o["obs"] for o in outs]),
             reward=np.array([o["reward"] for o in outs]), term=np.array([o["term"] for o in outs]),
             dbl=np.stack([o["dbl"] for o in outs]), ints=np.stack([o["ints"] for o in outs]),
             rng=np.stack([o["rng"] for o in outs]), **extra)
    json.dump(dict(info=[o["info"] for o in outs]), open(f[:-4] + ".json", "w"))


def _parse(spec):
    f = spec.split(",")
    A, K, T, seed = (int(x) for x in f[:4])
    env_class = f[4] if len(f) > 4 and f[4] else "AllFullRLProgressRewardEnv"
    otol = float(f[5]) if len(f) > 5 and f[5] else 0.0
    return A, K, T, seed, env_class, otol


def _make(spec):
    A, K, T, seed, env_class, otol = _parse(spec)
    t0 = time.time()
    load_traj(A, K, T, seed, env_class, oracle_tol=otol)
    return f"{spec}: {time.time() - t0:.1f} s"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--tol", type=float, default=0.0)
    ap.add_argument("--iters", type=int, default=0)
    ap.add_argument("--tag", default="")
    ap.add_argument("--traj", nargs="*", default=["2,4,96,7", "2,4,300,21", "2,8,300,5", "2,10,250,9"])
    ap.add_argument("--make-only", action="store_true", help="oracle rollouts into the cache only (no GPU)")
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--verbose-tol", type=float, default=None, help="print the worst entry of steps above this")
    args = ap.parse_args()
    po.build()
    if args.make_only:
        # tight trajectories first (the tolerance variants restep their states)
        specs = sorted(set(args.traj), key=lambda s: len(s.split(",")))
        import multiprocessing as mp
        with mp.get_context("fork").Pool(max(1, args.workers)) as pool:
            tight = sorted({",".join(s.split(",")[:4] + [s.split(",")[4]] if len(s.split(",")) > 4 and s.split(",")[4]
                                     else s.split(",")[:4]) for s in specs})
            for out in pool.imap_unordered(_make, tight):
                print(out, flush=True)
            for out in pool.imap_unordered(_make, [s for s in specs if len(s.split(",")) > 5]):
                print(out, flush=True)
        return
    for spec in args.traj:
        A, K, T, seed, env_class, otol = _parse(spec)
        t0 = time.time()
        traj = load_traj(A, K, T, seed, env_class, oracle_tol=otol)
        t1 = time.time()
        r = pu.compare(traj, args.prec, A, K, env_class, verbose_tol=args.verbose_tol, solver_tolerance=args.tol,
                       solver_iterations=args.iters)
        s = pu.summary(r)
        s.update(tag=args.tag, lib=os.path.basename(os.environ.get("FACTORYSIM_LIB", "libfactorysim.so")),
                 prec=args.prec, tol=args.tol,
                 traj=spec, rollout_s=round(t1 - t0, 1), gpu_s=round(time.time() - t1, 1))
        print(json.dumps(s), flush=True)


if __name__ == "__main__":
    main()
