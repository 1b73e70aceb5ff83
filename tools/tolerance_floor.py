#!/usr/bin/env python3
"""What MuJoCo's own Newton tolerance costs against the parity gate (test infrastructure, CPU).

The oracle sits at the solver's optimum (tolerance 1e-12).  This study steps, from every state of the same
teacher-forced trajectories the GPU sweep uses, a second float64 oracle whose Newton stops at tolerance TOL (MuJoCo's
default opt.tolerance is 1e-8) and reports the fraction of env-steps within the SURVEY gate -- i.e. how far a float64
MuJoCo-like solve at that tolerance already sits from the optimum.

usage: python tools/tolerance_floor.py [TOL] [A K T seed ...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import pyoracle as po  # noqa: E402  (checker)
import fp32_floor as ff  # noqa: E402


def study(tol, A, K, T, seed_actions):
    rng = np.random.default_rng(seed_actions)
    e = po.Env(A, K, 42, reward="progress", weights=(0.2, 0.4, 0.1, 0.4))
    e.reset()
    p = po.Env(A, K, 42, reward="progress", weights=(0.2, 0.4, 0.1, 0.4))
    p.reset()
    L = po.lib()
    out = []
    for t in range(T):
        d, i, r = e.export_state()
        a = rng.uniform(-2, 2, 8 * A).astype(np.float32)
        p.import_state(d, i, r)
        L.or_set_solver_tol(0.0)
        _, _, term, _, info = e.step(a)
        L.or_set_solver_tol(tol)
        _, _, pterm, _, _ = p.step(a)
        L.or_set_solver_tol(0.0)
        d2, i2, _ = e.export_state()
        p2, pi2, _ = p.export_state()
        flip = (term != pterm) or not np.array_equal(i2, pi2)
        out.append(dict(step=t, err=None if term else ff.rel_err(A, K, p2, d2), term=bool(term), flip=bool(flip),
                        ncubes=int(info["num_obj"])))
        if term:
            e.reset()
    return out


def make_traj(tol, A, K, T, seed_actions, cache):
    """the parity sweep's trajectory (parity_util.rollout: states and actions of the 1e-12 oracle) with the
    expected outputs of the tolerance-`tol` oracle stepped from each state"""
    import parity_util as pu

    recs, acts, outs = pu.restep_at_tolerance(po, A, K, pu.rollout(po, A, K, T, seed_actions=seed_actions), tol)
    f = os.path.join(cache, f"traj_{A}_{K}_{T}_{seed_actions}_tol{tol:g}.npz")
    np.savez(f, recs=recs, acts=acts, obs=np.stack([o["obs"] for o in outs]),
             reward=np.array([o["reward"] for o in outs]), term=np.array([o["term"] for o in outs]),
             dbl=np.stack([o["dbl"] for o in outs]), ints=np.stack([o["ints"] for o in outs]),
             rng=np.stack([o["rng"] for o in outs]))
    json.dump(dict(info=[o["info"] for o in outs]), open(f[:-4] + ".json", "w"))
    return f


if __name__ == "__main__":
    args = sys.argv[1:]
    if "--make-traj" in args:
        args.remove("--make-traj")
        tol = float(args[0]) if args else 1e-8
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        po.build()
        cache = os.environ.get("FM_TRAJ_CACHE", os.path.join(ROOT, "traj_cache"))
        for A, K, T, sa in [(2, 4, 96, 7), (2, 4, 300, 21), (2, 8, 300, 5), (2, 10, 250, 9)]:
            print(make_traj(tol, A, K, T, sa, cache), flush=True)
        sys.exit(0)
    tol = float(args[0]) if args else 1e-8
    rest = [int(x) for x in args[1:]]
    trajs = [tuple(rest[i:i + 4]) for i in range(0, len(rest), 4)] or [(2, 4, 96, 7), (2, 4, 300, 21),
                                                                        (2, 8, 300, 5), (2, 10, 250, 9)]
    po.build()
    for A, K, T, sa in trajs:
        s = ff.summarize(study(tol, A, K, T, sa))
        print(json.dumps(dict(tol=tol, traj=f"{A},{K},{T},{sa}", **s)), flush=True)
