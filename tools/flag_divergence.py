#!/usr/bin/env python3
"""Flag / integer-state divergence rate over many random episodes (SURVEY.md §8(d) parity gates; test infra).

Rolls out N_EP episodes of the oracle (AllFullRL, random U[-1,1] actions like bench.py, each episode from reset
with its own action seed, until termination or --cap env-steps) on a process pool, then teacher-forces the GPU
from every recorded state (chunks of --chunk arenas per launch) and compares, per env-step: terminated /
out_of_reach / force_terminate, the integer task state (in-scene list, FIFO, counters, scores, RNG) and the
SURVEY state gate.  Prints one JSON line per precision.

usage: python tools/flag_divergence.py [--episodes 1000] [--cap 400] [--workers 16] [--prec fp32 fp64]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _episodes(args):
    first, count, A, K, cap = args
    from oracle import pyoracle as po  # checker
    from factory_marl_amd import state as st

    recs, acts, terms, oor, frc, ints, rngs, dbls, ep_of = [], [], [], [], [], [], [], [], []
    for ep in range(first, first + count):
        rng = np.random.default_rng(100_000 + ep)
        e = po.Env(A, K, 42, weights=(0.2, 0.4, 0.1, 0.4))
        e.reset()
        for t in range(cap):
            d, i, r = e.export_state()
            recs.append(st.pack(A, K, d, i, r))
            a = rng.uniform(-1, 1, 8 * A).astype(np.float32)
            _, _, term, _, info = e.step(a)
            d2, i2, r2 = e.export_state()
            acts.append(a)
            terms.append(term)
            oor.append(info["out_of_reach"])
            frc.append(info["force_terminate"])
            ints.append(i2)
            rngs.append(r2)
            dbls.append(d2)
            ep_of.append(ep)
            if term:
                break
    return (np.stack(recs), np.stack(acts), np.array(terms), np.array(oor), np.array(frc), np.stack(ints),
            np.stack(rngs), np.stack(dbls), np.array(ep_of))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=1000)
    ap.add_argument("--cap", type=int, default=400)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=16384)
    ap.add_argument("--prec", nargs="*", default=["fp32", "fp64"])
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=4)
    a = ap.parse_args()
    A, K = a.arms, a.objects
    from oracle import pyoracle as po

    po.build()
    t0 = time.time()
    per = max(1, a.episodes // (a.workers * 16))  # short jobs: a progress line every ~minute
    jobs = [(s, min(per, a.episodes - s), A, K, a.cap) for s in range(0, a.episodes, per)]
    parts = []
    with mp.get_context("fork").Pool(a.workers) as pool:
        for i, part in enumerate(pool.imap(_episodes, jobs)):  # progress lines keep a long rollout visibly alive
            parts.append(part)
            print(f"oracle rollout: {i + 1}/{len(jobs)} jobs, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    cat = [np.concatenate([p[k] for p in parts]) for k in range(9)]
    recs, acts, terms, oor, frc, ints, rngs, dbls, ep_of = cat
    t_roll = time.time() - t0
    n = len(recs)
    print(f"oracle: {a.episodes} episodes, {n} env-steps, {int(terms.sum())} terminations in {t_roll:.0f} s",
          file=sys.stderr, flush=True)
    import torch

    import parity_util as pu
    from factory_marl_amd import state as st

    nq, nv, nu, nd, ni = st.sizes(A, K)
    for prec in a.prec:
        t1 = time.time()
        flag = {"terminated": 0, "out_of_reach": 0, "force_terminate": 0}
        int_bad = 0
        within = 0
        compared = 0
        eps_bad = set()
        for lo in range(0, n, a.chunk):
            hi = min(n, lo + a.chunk)
            env = pu.gpu_env(hi - lo, prec, A, K)
            env.set_state(recs[lo:hi])
            _, _, term, _ = env.step_tensors(torch.as_tensor(acts[lo:hi], device=env.device))
            env.sync()
            got = env.get_state()
            gterm = term.cpu().numpy().astype(bool)
            goor = env.out_of_reach.cpu().numpy().astype(bool)
            gfrc = env.force_terminate.cpu().numpy().astype(bool)
            env.close()
            for j in range(hi - lo):
                s = lo + j
                bad = False
                if gterm[j] != terms[s]:
                    flag["terminated"] += 1
                    bad = True
                if goor[j] != oor[s]:
                    flag["out_of_reach"] += 1
                    bad = True
                if gfrc[j] != frc[s]:
                    flag["force_terminate"] += 1
                    bad = True
                if terms[s]:
                    if bad:
                        eps_bad.add(int(ep_of[s]))
                    continue
                gd, gi, gr = st.unpack(A, K, got[j])
                if not (np.array_equal(gi[:2 * K + 10], ints[s][:2 * K + 10]) and np.array_equal(gr, rngs[s])):
                    int_bad += 1
                    bad = True
                qd, vd = pu.state_err(A, K, gd, dbls[s])
                within += int(max(qd.max(), vd.max()) <= 1e-4)
                compared += 1
                if bad:
                    eps_bad.add(int(ep_of[s]))
        out = dict(precision=prec, A=A, K=K, episodes=a.episodes, env_steps=int(n), terminations=int(terms.sum()),
                   force_terminations=int(frc.sum()), out_of_reach=int(oor.sum()),
                   flag_divergences=flag, flag_divergence_rate=round(sum(flag.values()) / n, 7),
                   int_state_divergences=int_bad, int_state_divergence_rate=round(int_bad / max(compared, 1), 7),
                   episodes_with_any_divergence=len(eps_bad), within_survey_gate=round(within / max(compared, 1), 5),
                   oracle_rollout_s=round(t_roll, 1), gpu_compare_s=round(time.time() - t1, 1),
                   note="teacher forcing: every recorded oracle state stepped once on the GPU with the oracle's action")
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
