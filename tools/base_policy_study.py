#!/usr/bin/env python3
"""IK base policy under the report's evaluation protocol, with a per-arm breakdown (test infrastructure: the oracle,
the CPU restatement the GPU kernel is parity-tested against, fp64).

Protocol (/root/reference/src/visualisation.py:55-80, report.tex:276-295): one FactoryManipulationEnv (every arm on
its IKPolicy), scene / TaskManager seed 42, K = 10 objects, E sequential episodes -- env.reset() after each
termination, the TaskManager RNG running on --, episode length = the 0-based index t of the terminating step,
scores = info["scores"] at termination.  Per arm, from the IKPolicy FSM (ik_policy.py:174-250) read after every
env-step: entries into each state, lost grasps (POST_GRASP / GO_TO_RELEASE -> IDLE before RELEASE), timeouts (the
state counter passing timeout_steps, ik_policy.py:249-250), and the IK solves that did not converge (act() then
returns last_ctrl, ik_policy.py:266-267); per episode the termination cause.

usage: python tools/base_policy_study.py [--arms 2] [--episodes 100] [--objects 10] > profiles/r04_base_policy.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle as po  # noqa: E402  (checker / study tool)

STATES = po.IK_STATES


def _stats(x):
    x = np.asarray(x, np.float64)
    return dict(mean=float(x.mean()), se=float(x.std(ddof=1) / np.sqrt(len(x))) if len(x) > 1 else 0.0, n=int(len(x)))


def study(A, K, episodes, seed=42):
    po.build()
    e = po.Env(A, K, seed, env_class="FactoryManipulationEnv")
    e.reset()
    timeout = 30  # ik_policy.py:67 at the default control frequency (3 s / 0.1 s)
    per_arm = [dict(entries={s: 0 for s in STATES}, lost_grasp=0, timeouts=0, timeouts_in={s: 0 for s in STATES})
               for _ in range(A)]
    prev = [e.ik_arm(i) for i in range(A)]
    eps = []
    t = 0
    t0 = time.time()
    while len(eps) < episodes:
        _, _, term, _, info = e.step(np.zeros(0, np.float32))
        cur = [e.ik_arm(i) for i in range(A)]
        for i in range(A):
            a, b = prev[i], cur[i]
            if b["state"] != a["state"]:
                per_arm[i]["entries"][STATES[b["state"]]] += 1
                if b["state"] == 0 and STATES[a["state"]] in ("POST_GRASP", "GO_TO_RELEASE"):
                    per_arm[i]["lost_grasp"] += 1
            if b["state"] == 0 and a["state"] != 0 and a["counter"] + 1 > timeout:
                per_arm[i]["timeouts"] += 1
                per_arm[i]["timeouts_in"][STATES[a["state"]]] += 1
        prev = cur
        if term:
            eps.append(dict(scores=info["scores"], length_t=t, out_of_reach=info["out_of_reach"],
                            force_terminate=info["force_terminate"]))
            e.reset()
            prev = [e.ik_arm(i) for i in range(A)]
            t = 0
            if len(eps) % 10 == 0:
                print(f"{len(eps)} episodes, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
        else:
            t += 1
    for i in range(A):
        calls, fails = e.ik_solve_counts(i)
        per_arm[i].update(ik_solves=calls, ik_failures=fails, bucket=i % 2)
    sc = np.array([x["scores"] for x in eps])
    return dict(protocol="visualisation.py:55-80: one env, seed 42, sequential episodes, TaskManager RNG running on",
                A=A, K=K, episodes=len(eps), seconds=round(time.time() - t0, 1),
                scores0=_stats(sc[:, 0]), scores1=_stats(sc[:, 1]), length_t=_stats([x["length_t"] for x in eps]),
                terminations=dict(out_of_reach=int(sum(x["out_of_reach"] for x in eps)),
                                  force=int(sum(x["force_terminate"] for x in eps))),
                per_arm=per_arm,
                reference_report={2: dict(scores=(1.65, 1.17), length=208.8),
                                  4: dict(scores=(1.18, 1.16), length=119.74)}.get(A))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=10)
    ap.add_argument("--episodes", type=int, default=100)
    args = ap.parse_args()
    print(json.dumps(study(args.arms, args.objects, args.episodes), indent=1))


if __name__ == "__main__":
    main()
