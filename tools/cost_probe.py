#!/usr/bin/env python3
"""Load balance of the config-2 launch (GPU box): each arena's env-step duration (fm_get_costs), the step's Newton
iterations and reruns per arena, then a list-scheduling replay of the measured durations over the launch's wave slots
-- perfect longest-first, longest-first by the previous step's durations (what lpt_order_kernel does), plain order.

usage: python tools/cost_probe.py [--steps 16] [--slots 2048] [--out profiles/r04o_cost_replay.json]
"""
import argparse
import heapq
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def makespan(order, cost, slots):
    """greedy list scheduling: each arena in `order` starts on the first free slot"""
    h = [0.0] * slots
    for i in order:
        t = heapq.heappop(h)
        heapq.heappush(h, t + cost[i])
    return max(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arenas", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--slots", type=int, default=2048, help="resident arenas: 256 CUs x 8 at (2,4) fp32")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    import bench
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    N = a.arenas
    env = FactoryVecEnv(N, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42),
                        precision="fp32", return_numpy=False)
    env.reset()
    bench.preroll(env, 200, 0, env.device)
    g = torch.Generator(device=env.device)
    g.manual_seed(0)
    costs, ms, reruns, newton, contacts, objs = [], [], [], [], [], []
    for _ in range(a.steps):
        act = bench.random_actions(env, torch.rand(N, env.act_dim, device=env.device, generator=g))
        c0 = env.counters()
        env.sync()
        t0 = time.perf_counter()
        env.step_tensors(act)
        env.sync()
        ms.append((time.perf_counter() - t0) * 1e3)
        d = env.counters() - c0
        reruns.append(int(d[:, 8].sum()))
        newton.append(d[:, 1].astype(np.float64))
        contacts.append(d[:, 4].astype(np.float64))  # contacts demanded, summed over the step's stages
        objs.append(d[:, 6].astype(np.float64))  # objects in scene at the step's end
        costs.append(env.costs().astype(np.float64) / 1e5)  # 100 MHz wall clock -> ms
    env.close()
    rows = []
    for k in range(1, a.steps):
        cur = costs[k]
        rows.append(dict(step=k, measured_ms=round(ms[k], 2), reruns=reruns[k], mean_cost_ms=round(float(cur.mean()), 3),
                         max_cost_ms=round(float(cur.max()), 2), p99_cost_ms=round(float(np.quantile(cur, 0.99)), 2),
                         lpt_perfect_ms=round(makespan(np.argsort(-cur), cur, a.slots), 2),
                         lpt_prev_order_ms=round(makespan(np.argsort(-costs[k - 1]), cur, a.slots), 2),
                         plain_order_ms=round(makespan(np.arange(N), cur, a.slots), 2),
                         corr_prev_cost=round(float(np.corrcoef(costs[k - 1], cur)[0, 1]), 3),
                         corr_newton_iters=round(float(np.corrcoef(newton[k], cur)[0, 1]), 3),
                         # intrinsic-work predictors from the previous step's counters (a duration also carries the
                         # co-scheduled wave's load): longest-first by them, and their correlation with this step's cost
                         lpt_prev_newton_ms=round(makespan(np.argsort(-newton[k - 1]), cur, a.slots), 2),
                         lpt_prev_contacts_ms=round(makespan(np.argsort(-contacts[k - 1]), cur, a.slots), 2),
                         lpt_prev_objects_ms=round(makespan(np.argsort(-objs[k - 1], kind="stable"), cur, a.slots), 2),
                         corr_contacts=round(float(np.corrcoef(contacts[k], cur)[0, 1]), 3),
                         corr_prev_contacts=round(float(np.corrcoef(contacts[k - 1], cur)[0, 1]), 3),
                         corr_prev_newton=round(float(np.corrcoef(newton[k - 1], cur)[0, 1]), 3)))
    rep = dict(source="tools/cost_probe.py: config-2 workload (4096 arenas (2,4) fp32, 200-step pre-roll), fm_get_costs "
                      "after each step; list-scheduling replay over %d wave slots" % a.slots, steps=rows)
    txt = json.dumps(rep, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
