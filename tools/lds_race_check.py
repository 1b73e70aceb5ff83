#!/usr/bin/env python3
"""LDS race and bounds check of the env-step kernels on the CPU backend (test/measurement infra, CPU only).

The kernel's lanes hand data to each other through LDS at SYNC() (fm_device.hpp).  On the GPU one wave executes in
lockstep, so a hand-off that lacks the barrier still works there; the CPU backend runs the 64 lanes of a wave one
after another between cross-lane points (fm_simt_host.hpp), where it does not.  This tool runs the CPU backend built
with the race detector (fm_cpu.cpp FM_RACE_DETECT: the TSan instrumentation hooks, a shadow word per 4 bytes of LDS)
over a few env-steps of each case and prints every pair of source lines where two lanes touched the same LDS
word between two rendezvous with at least one write (RAW / WAR / WAW), symbolized with llvm-symbolizer, and every
out-of-bounds access: LDS past the arena's workspace (LDS-OOB: the emulated LDS has guard zones) and global scratch
outside the arena's own block (SCRATCH-OOB); an array index past a local array's bound traps (UBSan, SIGILL: the
CPU backend's FACTORYSIM_CPU_TRACE report names the lane and block).

Since round 6 the CPU backend runs the compile-time scene kernels (fm_cpu_fixed.cpp) -- the code the GPU benchmarks
run: the (2,4) 64-contact kernel and its float64 wide rerun, the spill layouts of (2,8), (2,10), (4,16), the cached
midphase, arrowhead / tree-block / matrix-core factors.  The rerun cases need the experiment switches (FM_FORCE_RERUN,
FM_RERUN_AT_50): build the detector library with them.

usage: make -C factory_marl_amd/csrc race OBJDIR=build_race XDEFS=-DFM_EXPERIMENTS=1   (builds scratch/lib_race.so)
       FACTORYSIM_LIB=scratch/lib_race.so python tools/lds_race_check.py
       [RACE_STEPS=n] [RACE_CASES=i,j] [RACE_PRECISIONS=fp64,fp32]   (a case takes minutes: run cases in parallel)
       [RACE_TRAJ=A,K,T,seed,EnvClass [RACE_PICK=lo:hi]]   (a parity test's teacher-forced launch instead)"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.environments import run_kwargs

    # (env class, A, K, experiment switches): the switches need the experiment build (FM_EXPERIMENTS=1)
    cases = [("AllFullRLProgressRewardEnv", 2, 4, ""), ("PauseIKToggleEnv", 2, 4, ""), ("AllDeltaProgressRewardEnv", 2, 4, ""),
             ("AllFullRLProgressRewardEnv", 2, 8, ""), ("AllFullRLProgressRewardEnv", 2, 10, ""),
             ("PauseIKToggleEnv", 4, 16, ""), ("AllFullRLProgressRewardEnv", 2, 4, "FM_FORCE_RERUN=1"),
             ("AllFullRLProgressRewardEnv", 2, 4, "FM_RERUN_AT_50=1"), ("PauseIKToggleEnv", 2, 4, "FM_FORCE_RERUN=1"),
             ("AllFullRLProgressRewardEnv", 2, 8, "FM_NO_TREEBLK=1"), ("BackupIKToggleEnv", 2, 10, ""),
             ("PauseIKToggleEnv", 2, 10, ""), ("BackupIKToggleEnv", 2, 8, "")]
    steps = int(os.environ.get("RACE_STEPS", "3"))
    if os.environ.get("RACE_TRAJ"):
        # A,K,T,seed,EnvClass: the records of an oracle rollout stepped teacher-forced in one launch (a GPU parity
        # test's launch, e.g. one that faulted on the GPU)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import parity_util as pu
        from oracle import pyoracle

        pyoracle.build()
        sp = os.environ["RACE_TRAJ"].split(",")
        A_, K_, T_, seed = map(int, sp[:4])
        tr = pu.rollout(pyoracle, A_, K_, T_, seed_actions=seed, env_class=sp[4])
        pick = os.environ.get("RACE_PICK")  # a subset of the records: lo:hi
        if pick:
            lo, hi = map(int, pick.split(":"))
            tr = tuple(x[lo:hi] for x in tr)
        for prec in os.environ.get("RACE_PRECISIONS", "fp32").split(","):
            s = pu.summary(pu.compare(tr, prec, A_, K_, sp[4], device="cpu"))
            print(f"ran {prec} {sp[4]} ({A_},{K_}) teacher-forced x {len(tr[0])}: within {s['within']}, worst "
                  f"{s['worst']:.2e}", flush=True)
        cases = []
    if os.environ.get("RACE_CASES"):
        cases = [cases[int(i)] for i in os.environ["RACE_CASES"].split(",")]
    for prec in os.environ.get("RACE_PRECISIONS", "fp64,fp32").split(",") if cases else []:
        for cls, A, K, exp in cases:
            env = FactoryVecEnv(1, env_class=cls, env_kwargs=run_kwargs(cls, num_arms=A, max_num_objects=K, seed=42),
                                device="cpu", precision=prec, experimental=bool(exp))
            if exp:
                env.set_experiment(exp)
            env.reset()
            rng = np.random.default_rng(0)
            for _ in range(steps):
                if cls in ("PauseIKToggleEnv", "BackupIKToggleEnv"):
                    a = (rng.random((1, env.act_dim)) < 0.5).astype(np.float32)
                else:
                    a = rng.uniform(-1, 1, (1, env.act_dim)).astype(np.float32)
                env.step(a)
            env.close()
            print(f"ran {prec} {cls} ({A},{K}) {exp} x {steps}", flush=True)
    lib = os.environ["FACTORYSIM_LIB"]
    L = C.CDLL(lib)
    buf = C.create_string_buffer(1 << 20)
    n = L.fm_race_report(buf, len(buf))
    text = buf.value.decode().split("\n", 1)
    lay = [int(x) for x in text[0].split()[1:]]
    lines = text[1].split()
    print(f"{n} racing access pairs")
    kinds = {"0": "RAW", "1": "WAR", "2": "WAW", "3": "LDS-OOB", "4": "SCRATCH-OOB"}
    recs = [(kinds[lines[i]], lines[i + 1], lines[i + 2], int(lines[i + 3])) for i in range(0, len(lines), 4)]
    names = lay_names()
    sym = os.path.join("/opt/rocm/lib/llvm/bin", "llvm-symbolizer")
    allpc = sorted({pc for _, a, b, _ in recs for pc in (a, b) if int(pc, 16) > 0})
    out = subprocess.run([sym, "--obj", lib, "--inlining", "--functions=short"] + allpc, capture_output=True,
                         text=True).stdout
    blocks = [b.strip().splitlines() for b in out.strip().split("\n\n")]

    def site(blk):
        # (function, file:line) pairs innermost first; an optimised-away line (":0:") takes its caller's line
        frames = [(blk[i], blk[i + 1].split("csrc/")[-1]) for i in range(0, len(blk) - 1, 2)]
        for fn, loc in frames:
            if ":0:" not in loc:
                return f"{loc} ({fn})"
        return frames[0][1] if frames else "?"

    where = {pc: site(blk) for pc, blk in zip(allpc, blocks)}
    where.update({pc: "-" for _, a, b, _ in recs for pc in (a, b) if int(pc, 16) <= 0})
    seen = set()
    for kind, a, b, off in recs:
        k = (kind, where[a], where[b])
        if k in seen:
            continue
        seen.add(k)
        print(f"{kind}: {where[a]}  <->  {where[b]}   [{region(off, names, lay, kind)}]")


def lay_names():
    """the int fields of struct Lay (fm_dev.hpp), in order"""
    import re
    src = open(os.path.join(ROOT, "factory_marl_amd/csrc/fm_dev.hpp")).read()
    body = src[src.index("struct Lay {") + 12:]
    body = body[:body.index("};")]
    body = re.sub(r"//[^\n]*", "", body)
    return [n.strip() for decl in body.split(";") if decl.strip().startswith("int ")
            for n in decl.strip()[4:].split(",")]


def region(off, names, lay, kind=""):
    if kind == "SCRATCH-OOB":
        return f"scratch buffer +{off}"
    if kind == "LDS-OOB":
        return f"LDS {off:+d} (workspace {lay[-3] if lay else '?'} B)"
    if off < 0:
        return "global"
    if not lay:
        return f"LDS +{off}"
    best = max(((v, n) for n, v in zip(names, lay) if 0 <= v <= off), default=(0, "?"))
    return f"LDS +{off} = {best[1]} +{off - best[0]}"


if __name__ == "__main__":
    main()
