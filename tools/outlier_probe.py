#!/usr/bin/env python3
"""What makes the config-2 launch's slowest arenas slow (GPU box; measurement infra).

With the longest-first order the launch's makespan is set by its slowest arena whenever that arena's env-step takes
longer than the launch's other work (round 5, profiles/r05k_cost_replay.json: mean arena env-step 5.9 ms, 99th
percentile 7.5 ms, maximum 13-20 ms; the replay with perfect knowledge equals the maximum in most steps).  This probe
runs the config-2 workload, keeps the records and actions of the costliest arenas (fm_get_costs) and of median ones
over a few steps, then replays each group -- every record copied to fill a 4096-arena launch, so the occupancy is the
benchmark's -- with the phase profiler on (fm_profile), and reports per group: env-step duration, Newton iterations,
contacts, objects, and the per-phase wall time per arena-substep.

usage: python tools/outlier_probe.py [--steps 12] [--top 16] [--out profiles/r06_outliers.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_env(n, precision):
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    return FactoryVecEnv(n, env_kwargs=run_kwargs("AllFullRLProgressRewardEnv", num_arms=2, max_num_objects=4, seed=42),
                         precision=precision, return_numpy=False)


def replay(recs, acts, n, precision):
    """one env-step of `n` arenas holding copies of the records, profiled; per-phase us per arena-substep"""
    import torch

    env = make_env(n, precision)
    env.reset()
    k = len(recs)
    idx = np.arange(n) % k
    env.set_state(recs[idx])
    a = torch.as_tensor(acts[idx], device=env.device)
    env.step_tensors(a)  # warm (the compile / first-launch costs), then the profiled step from the same records
    env.sync()
    env.set_state(recs[idx])
    c0 = env.counters()
    env.profile(1)
    env.step_tensors(a)
    env.sync()
    ph, ncon = env.profile(0)
    c1 = env.counters()
    cost = env.costs().astype(np.float64) / 100.0  # s_memrealtime ticks at 100 MHz -> us
    env.close()
    sub = n * 100
    d = c1 - c0
    per_rec = np.array([cost[idx == j].mean() for j in range(k)]) / 1e3
    return {"record_cost_ms_top": [round(float(x), 3) for x in np.sort(per_rec)[::-1][:8]],
            "record_cost_ms_p50": round(float(np.median(per_rec)), 3),"phases_us_per_arena_substep": {kk: round(v / sub * 1e6, 3) for kk, v in sorted(ph.items())},
            "total_us_per_arena_substep": round(sum(ph.values()) / sub * 1e6, 3),
            "env_step_ms_mean": round(float(cost.mean()) / 1e3, 3), "env_step_ms_max": round(float(cost.max()) / 1e3, 3),
            "newton_iters_per_substep": round(float(d[:, 1].sum()) / sub, 3),
            "contacts_per_substep": round(float(d[:, 4].sum()) / sub, 3), "max_contacts": int(c1[:, 5].max()),
            "objects": round(float(d[:, 6].sum()) / n, 3), "reruns": int(d[:, 8].sum()), "mean_ncon_profile": round(ncon / sub, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arenas", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--top", type=int, default=16)
    ap.add_argument("--preroll", type=int, default=200)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--solo", type=int, default=256, help="arenas of the uncontended replay (one per CU)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    import bench

    env = make_env(a.arenas, a.precision)
    env.reset()
    bench.preroll(env, a.preroll, 0, env.device)
    g = torch.Generator(device=env.device)
    g.manual_seed(0)
    rows, recs, acts = [], [], []
    for s in range(a.steps):
        s0 = env.get_state()
        act = torch.rand(a.arenas, env.act_dim, device=env.device, generator=g) * 2 - 1
        c0 = env.counters()
        env.step_tensors(act)
        env.sync()
        cost = env.costs().astype(np.float64) / 100.0
        d = env.counters() - c0
        an = act.cpu().numpy()
        order = np.argsort(cost)
        for i in list(order[-a.top:]) + list(order[len(order) // 2 - a.top // 2:len(order) // 2 + a.top // 2]):
            rows.append(dict(step=s, arena=int(i), cost_ms=float(cost[i]) / 1e3, newton=int(d[i, 1]),
                             contacts=int(d[i, 4]), objects=int(d[i, 6]), rerun=int(d[i, 8]),
                             top=bool(i in order[-a.top:])))
            recs.append(s0[i])
            acts.append(an[i])
        print(f"step {s}: mean {cost.mean() / 1e3:.2f} ms, p99 {np.quantile(cost, 0.99) / 1e3:.2f}, max "
              f"{cost.max() / 1e3:.2f}", file=sys.stderr, flush=True)
    env.close()
    recs, acts = np.stack(recs), np.stack(acts)
    top = np.array([r["top"] for r in rows])
    out = {"source": "tools/outlier_probe.py: config-2 workload, fm_get_costs per arena; each group replayed in a "
                     f"{a.arenas}-arena launch of copies with fm_profile",
           "groups": {}}
    for name, m in (("slowest", top), ("median", ~top)):
        rr = [r for r, t in zip(rows, m) if t]
        out["groups"][name] = {
            "arenas": len(rr),
            "measured_cost_ms_mean": round(float(np.mean([r["cost_ms"] for r in rr])), 3),
            "measured_newton_iters_per_substep": round(float(np.mean([r["newton"] for r in rr])) / 100, 3),
            "measured_contacts_per_substep": round(float(np.mean([r["contacts"] for r in rr])) / 100, 3),
            "measured_objects": round(float(np.mean([r["objects"] for r in rr])), 3),
            "replay": replay(recs[m], acts[m], a.arenas, a.precision),
            # the same records alone on their SIMDs (one arena per CU): the env-step latency without a co-resident wave
            "replay_solo": replay(recs[m], acts[m], a.solo, a.precision)}
    out["rows"] = rows
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)


if __name__ == "__main__":
    main()
