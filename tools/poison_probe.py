#!/usr/bin/env python3
"""Uninitialised-read probe of the env-step kernels on the CPU backend (test/measurement infra, CPU only).

A kernel that reads a register, LDS word or scratch-block word before writing it sees whatever the previous user left
there on the GPU -- harmless by accident under one register allocation, a wrong value (or a wild address) under
another.  The CPU backend built at -O0 (every local on the emulated lane's fiber stack) can make such reads visible:
FACTORYSIM_CPU_POISON=<byte> fills the lanes' stacks, the emulated LDS and the arenas' global scratch blocks with that
byte before each workgroup runs.  This probe steps the same records once under several poison bytes, in separate
processes, and requires the resulting state records, observations, rewards and flags to be identical bit for bit:
any difference is a read of memory the kernel did not write first.  The -O0 build also keeps every branch of the
source as a branch, so a cross-lane operation (v_readlane, DPP, ballot, MFMA, barrier) reached by only part of the
wave -- legal on the GPU, where v_readlane ignores EXEC, but a dependence on how the compiler lays out the branch --
stops the emulator with both lanes' call chains.

usage: make -C factory_marl_amd/csrc OBJDIR=build_poison OUT=../../scratch/lib_poison.so HOSTOPT=-O0 SCENES=2_4
       python tools/poison_probe.py [--lib scratch/lib_poison.so] [--steps 96] [--pick 24]
           [--traj A,K,T,seed[,EnvClass]]   (a cached oracle trajectory, $FM_TRAJ_CACHE or traj_cache/)
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import parity_util as pu
d = np.load({inp!r})
out = {{}}
for prec in ("fp64", "fp32"):
    env = pu.gpu_env(len(d["recs"]), prec, {A}, {K}, device="cpu", env_class={cls!r})
    env.set_state(d["recs"])
    o, r, t, _ = env.step_tensors(torch.as_tensor(d["acts"]))
    out[prec + "_state"] = env.get_state()
    out[prec + "_obs"] = o.numpy().copy()
    out[prec + "_rew"] = r.numpy().copy()
    out[prec + "_term"] = t.numpy().copy()
    out[prec + "_tobs"] = env.terminal_obs.numpy().copy()
    out[prec + "_ctr"] = env.counters()
    env.close()
np.savez({outp!r}, **out)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "scratch", "lib_poison.so"))
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--pick", type=int, default=24)
    ap.add_argument("--poison", default="0,255,127")
    ap.add_argument("--env-class", default="AllFullRLProgressRewardEnv")
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=4)
    ap.add_argument("--traj", default=None, help="A,K,T,seed[,EnvClass]: records of a cached oracle trajectory")
    ap.add_argument("--crowded", action="store_true", help="the >64-contact (2,4) records (the wide rerun kernel)")
    a = ap.parse_args()
    import parity_util as pu
    from oracle import pyoracle

    pyoracle.build()
    A, K = a.arms, a.objects
    if a.crowded:
        # (2,4) records whose first stage holds 66-110 contacts: the 64-contact kernel abandons them, the float64 wide
        # kernel steps them (tests/test_gpu_parity.py::_crowded_trajectory)
        import test_gpu_parity

        recs, acts, outs = test_gpu_parity._crowded_trajectory(pyoracle)
        A, K = 2, 4
    elif a.traj:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import parity_sweep

        sp = a.traj.split(",")
        A, K, T, seed = map(int, sp[:4])
        a.env_class = sp[4] if len(sp) > 4 else "AllFullRLProgressRewardEnv"
        recs, acts, outs = parity_sweep.load_traj(A, K, T, seed, a.env_class,
                                                  cache=os.environ.get("FM_TRAJ_CACHE", os.path.join(ROOT, "traj_cache")))
    else:
        recs, acts, outs = pu.rollout(pyoracle, A, K, a.steps, seed_actions=7, env_class=a.env_class)
    # the records with the most contact work: every terminating step and an even spread over the rest
    idx = sorted(set([i for i, o in enumerate(outs) if o["term"]] +
                     list(np.linspace(0, len(recs) - 1, a.pick).astype(int))))
    tmp = tempfile.mkdtemp(prefix="poison_")
    inp = os.path.join(tmp, "in.npz")
    np.savez(inp, recs=recs[idx], acts=acts[idx])
    res = {}
    for pz in a.poison.split(","):
        outp = os.path.join(tmp, f"out_{pz}.npz")
        code = CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"), inp=inp, outp=outp, A=A, K=K,
                            cls=a.env_class)
        env = dict(os.environ, FACTORYSIM_LIB=a.lib, FACTORYSIM_CPU_POISON=pz, FACTORYSIM_CPU_THREADS="8")
        pr = subprocess.run([sys.executable, "-c", code], env=env, timeout=3000, capture_output=True, text=True)
        if pr.returncode != 0:
            print(json.dumps({"poison": pz, "returncode": pr.returncode, "stderr_tail": pr.stderr[-3000:]}))
            return 2
        res[pz] = dict(np.load(outp))
    base = res[a.poison.split(",")[0]]
    diff = {}
    for pz, r in res.items():
        for k, v in r.items():
            same = np.array_equal(v, base[k], equal_nan=True) if v.dtype.kind == "f" else np.array_equal(v, base[k])
            if not same:
                diff.setdefault(pz, []).append(k)
    rep = {"records": len(idx), "env_class": a.env_class, "scene": f"{A}x{K}", "poison_bytes": a.poison,
           "differences": diff, "identical": not diff}
    print(json.dumps(rep))
    return 0 if not diff else 1


if __name__ == "__main__":
    sys.exit(main())
