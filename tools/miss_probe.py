#!/usr/bin/env python3
"""Where a teacher-forced fp32 miss starts (test infrastructure; GPU box).  For chosen steps of a cached trajectory
(tools/parity_sweep.py load_traj): the kernel's first physics stage of the env-step (fm_debug_dump: contacts, M, bias,
qacc_smooth, the Newton solution qacc, qfrc_constraint) against the oracle's same stage (or_d_stage_fwd) from the
same record.  One JSON line per step: contact counts, worst matched-contact differences (dist, point, normal), and
the worst relative differences of qacc_smooth / qacc / qfrc_constraint with their dofs.

usage: python tools/miss_probe.py SPEC [--prec fp32] [--steps 23 71 101 ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import pyoracle as po  # noqa: E402  (checker)
from parity_sweep import _parse, load_traj  # noqa: E402


def rel(a, b, floor):
    d = np.abs(a - b) / np.maximum(np.abs(b), floor)
    j = int(np.argmax(d))
    return float(d[j]), j


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("spec")
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--steps", type=int, nargs="*", default=None)
    args = ap.parse_args()
    import parity_util as pu
    from factory_marl_amd import state as st

    po.build()
    L = po.lib()
    A, K, T, seed, env_class, _ = _parse(args.spec)
    recs, acts, outs = load_traj(A, K, T, seed, env_class)
    steps = args.steps if args.steps else list(range(0, len(recs), 10))
    env = pu.gpu_env(1, args.prec, A, K, env_class)
    e = po.Env(A, K, 42, weights=(0.2, 0.4, 0.1, 0.4), env_class=env_class)
    e.reset()
    m, dd = e.model, e.data
    nv = m.nv
    for s in steps:
        env.set_state(recs[s][None])
        g = env.debug_dump(0, actuated=True)
        d, i, r = st.unpack(A, K, recs[s])
        f = st.fields(A, K, d)
        dd.qpos[:] = f["qpos_stage"]
        dd.qvel[:] = f["qvel_stage"]
        dd.qacc_warmstart[:] = f["qacc_warmstart"]
        dd.ctrl[:] = f["ctrl_target"]
        L.or_d_stage_fwd(m.h, dd.h, 1)
        qs = np.ctypeslib.as_array(L.or_d_qacc_smooth(dd.h), shape=(nv,)).copy()
        cons = dd.contacts()
        ref = {}
        for c in cons:
            ref.setdefault(tuple(c["geom"]), []).append(c)
        worst = dict(dist=0.0, pos=0.0, normal=0.0)
        unmatched = 0
        seen = {}
        for c in g["con"]:
            key = (int(c[0]), int(c[1]))
            k = seen.get(key, 0)
            seen[key] = k + 1
            lst = ref.get(key, [])
            if k >= len(lst):
                unmatched += 1
                continue
            rc = lst[k]
            worst["dist"] = max(worst["dist"], abs(c[2] - rc["dist"]))
            worst["pos"] = max(worst["pos"], float(np.abs(c[3:6] - rc["pos"]).max()))
            worst["normal"] = max(worst["normal"], float(np.abs(c[6:9] - rc["frame"][0]).max()))
        out = dict(step=s, ncon_ref=int(dd.ncon), ncon_gpu=int(g["ncon"]), unmatched=unmatched, contact_worst=worst)
        for name, a_, b_, fl in [("qacc_smooth", g["as"], qs, 1.0), ("qacc", g["a"], dd.qacc, 1.0),
                                 ("qfrc_constraint", g["fc"], dd.qfrc_constraint, 1.0)]:
            v, j = rel(a_, b_, fl)
            out[name] = dict(rel=v, dof=pu.entry_name(A, K, 1 + 7 * K + 9 * A + j, d), ref=float(b_[j]),
                             got=float(a_[j]))
        print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
