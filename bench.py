#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the batched factory-manipulation env-step on MI355X.

Metric (BASELINE.json): env-steps/sec (whole node), 4096 arenas 2-arm x 4-obj, 1/2/4/8 MI355X.
Workload (BASELINE.md / SURVEY.md §8d, config 2): 4096 arenas per GPU, A=2 arms, K=4 cubes,
AllFullRLProgressRewardEnv, random policy U[-1,1]^16 drawn from a Philox stream (seed 0 + rank) before the
timed region (policy excluded), auto-reset inside the step.  One step = one env-step of every arena
(100 physics substeps + task layer).  Multi-GPU: one process per GPU (factory_marl_amd/launch.py), arenas
are independent (weak scaling, no data-path collective); value = all ranks' env-steps / max-over-ranks time.

Episode mix: all arenas start from reset in lockstep, so before timing every arena is pre-rolled with
random actions and reset once at a random offset (masked fm_reset) -- the timed window then holds arenas
at every episode phase (cube counts, contacts, terminations and auto-resets in their stationary mix,
reported under "diagnostics") instead of the first seconds of one synchronised episode.

Roofline: the dominant (only) kernel in the timed region is fm::step_kernel; its average launch time is
measured with HIP events on the stream it runs on.  Algorithmic bytes per arena env-step
B(A,K) = 100*8*(nq + 2nv + nu) + 4*(act_dim + obs_dim + 4) = 120,480 B at (2,4).  The
kernel is bound by neither HBM nor MFMA but by dependent LDS / VALU / L2 latency chains at two waves per SIMD;
"roofline.valu" prices its VALU work (PMC instruction counts per arena env-step, profiles/) against the
fp32 vector peak with the live kernel time.
CPU baseline: the oracle (our C restatement of the reference algorithm, oracle/) stepped with OpenMP on
the host cores of the same box, on a bounded sample, rank 0 at N=1 only.

Launch: ``python bench.py --gpus N`` starts N rank processes itself (the parent touches no GPU; RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* at 127.0.0.1, one GPU each) and prints rank 0's line; under torchrun (WORLD_SIZE set) the
process is one rank and --gpus must equal WORLD_SIZE.  --scaling weak (default): --arenas per GPU; strong: --arenas
is the job total, split over the ranks.  --workload config4: 131072 arenas (2,8) strong-split over the ranks with
the PPO rollout + RCCL update of config 3.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from factory_marl_amd.environments import run_kwargs  # noqa: E402
from factory_marl_amd.launch import (RankContext, arena_seeds, job_throughput, max_over_ranks,  # noqa: E402,F401
                                     rank_arenas)

HBM_PEAK_GBPS = 8000.0     # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
FP32_PEAK_TFLOPS = 157.3   # MI355X fp32 vector peak (same table)
FP64_PEAK_TFLOPS = 78.6    # fp64 vector rate = 1/2 of fp32


def algorithmic_bytes(A, K):
    nq, nv, nu = 1 + 7 * K + 9 * A, 1 + 6 * K + 9 * A, 1 + 8 * A
    obs_dim, act_dim = 24 * A + 13 * K, 8 * A
    return 100 * 8 * (nq + 2 * nv + nu) + 4 * (act_dim + obs_dim + 4)


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return "unknown"


def cpu_baseline(A, K, seconds):
    """oracle env-steps/s on the host cores (OpenMP), bounded sample"""
    import ctypes as C

    from oracle import pyoracle  # test infrastructure: the CPU baseline leg only

    pyoracle.build()
    L = pyoracle.lib()
    cores = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "64"))))
    # calibrate: one env-step per core first
    n = C.c_int64(0)
    dt = L.or_batch_bench(A, K, cores, 2, cores, 1, C.byref(n))
    rate = n.value / max(dt, 1e-9)
    steps = max(2, int(rate * seconds / cores))
    dt = L.or_batch_bench(A, K, cores, steps, cores, 0, C.byref(n))
    return {"value": round(n.value / dt, 3), "unit": "env-steps/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{cores} arenas x {steps} env-steps ({A} arms x {K} objects, random actions), "
                      f"oracle/ C restatement (fp64, OpenMP; static collision-pair list with body-level bounds, "
                      f"envelope Cholesky of M and the Newton Hessian, sparse constraint rows), {dt:.1f} s wall"}


def preroll(env, steps, rank, device):
    """desynchronise the arenas: random actions, each arena reset once at a random offset in [0, steps)"""
    import numpy as np
    import torch

    if steps <= 0:
        return
    N = env.num_envs
    off = np.random.default_rng(1234 + rank).integers(0, steps, N)
    g = torch.Generator(device=device)
    g.manual_seed(10_000 + rank)
    for s in range(steps):
        m = (off == s).astype(np.uint8)
        if m.any():
            env.reset(mask=m)
        env.step_tensors(random_actions(env, torch.rand(N, env.act_dim, device=device, generator=g)))


def random_actions(env, u):
    """random policy of the env class: U[-1, 1] Box actions, or fair-coin MultiDiscrete toggles (0.0 / 1.0)"""
    if env.env_class in ("PauseIKToggleEnv", "BackupIKToggleEnv"):
        return (u < 0.5).float()
    return u * 2.0 - 1.0


def timed_run(ctx, args, precision, steps, warmup, lo, hi):
    """build, pre-roll, warm up and time `steps` env-steps of this rank's arenas; returns (wall, kernel ms,
    counter deltas over the timed window)"""
    import torch

    from factory_marl_amd import FactoryVecEnv

    A, K, N = args.arms, args.objects, hi - lo
    env = FactoryVecEnv(N, env_class=args.env_class,
                        env_kwargs=run_kwargs(args.env_class, num_arms=A, max_num_objects=K, seed=42),
                        device=ctx.local_rank, precision=precision, seeds=arena_seeds(lo, hi, args.seeds),
                        solver_tolerance=args.solver_tolerance)
    env.reset()
    preroll(env, args.preroll, ctx.rank, ctx.device)
    g = torch.Generator(device=ctx.device)
    g.manual_seed(0 + ctx.rank)
    total = warmup + steps
    acts = random_actions(env, torch.rand(total, N, env.act_dim, device=ctx.device, generator=g, dtype=torch.float32))
    for s in range(warmup):
        env.step_tensors(acts[s])
    torch.cuda.synchronize()
    c0 = env.counters()
    env.kernel_timing(True)  # HIP event pair around each step-kernel launch, on the env's own stream
    ctx.barrier()
    t0 = time.perf_counter()
    for s in range(warmup, total):
        env.step_tensors(acts[s])
    ctx.barrier()
    wall = time.perf_counter() - t0
    k_ms, k_n = env.kernel_time()
    # average duration of the env-step kernel alone (fm_get_kernel_time): the region also holds the longest-first
    # order kernel, the rerun-list reset and the (2,4) wide rerun launch, which the event pairs leave out
    kern_ms = k_ms / max(k_n, 1)
    env.kernel_timing(False)
    c1 = env.counters()
    dc = c1 - c0
    dc[:, 5] = c1[:, 5]  # running maximum (contacts demanded by one stage), not a sum: keep the level
    env.close()
    return wall, kern_ms, dc


def timed_run_ppo(ctx, args, lo, hi):
    """config 3: PPO rollout with the PyTorch-ROCm policy ([128, 128] tanh MLPs, SB3 MlpPolicy) in the loop --
    policy forward, Gaussian sampling, clip, env-step, rollout-buffer writes are all inside the timed region;
    then one PPO update (GAE + n_epochs x minibatches) over the collected rollout, timed separately"""
    import torch

    from factory_marl_amd import FactoryVecEnv
    from factory_marl_amd.ppo import PPO

    A, K, N = args.arms, args.objects, hi - lo
    env = FactoryVecEnv(N, env_kwargs=run_kwargs(args.env_class, num_arms=A, max_num_objects=K, seed=42),
                        device=ctx.local_rank,
                        precision=args.precision, seeds=arena_seeds(lo, hi, args.seeds),
                        solver_tolerance=args.solver_tolerance)
    env.reset()
    preroll(env, args.preroll, ctx.rank, ctx.device)
    dist = None
    if ctx.world > 1:
        import torch.distributed as dist
    ppo = PPO(env, n_steps=args.steps, batch_size=args.ppo_batch, n_epochs=args.ppo_epochs, seed=ctx.rank, dist=dist)
    ppo._last_obs = env.obs.clone()
    ppo._last_starts = torch.zeros(N, device=ctx.device)
    ppo.hp["n_steps"] = args.warmup
    if args.warmup:
        ppo.collect_rollouts()
    ppo.hp["n_steps"] = args.steps
    torch.cuda.synchronize()
    c0 = env.counters()
    env.kernel_timing(True)  # HIP event pair around each step-kernel launch (the roofline's kernel time)
    ctx.barrier()
    t0 = time.perf_counter()
    buf, _ = ppo.collect_rollouts()
    torch.cuda.synchronize()
    ctx.barrier()
    wall = time.perf_counter() - t0
    k_ms, k_n = env.kernel_time()
    env.kernel_timing(False)
    kern_ms = k_ms / max(k_n, 1)
    c1 = env.counters()
    dc = c1 - c0
    dc[:, 5] = c1[:, 5]
    t1 = time.perf_counter()
    ppo.train(buf)
    torch.cuda.synchronize()
    ctx.barrier()
    train_s = time.perf_counter() - t1
    env.close()
    return wall, train_s, dc, kern_ms


def diagnostics(dc, N, steps, frame_skip=100):
    es = N * steps
    return {"env_steps_timed": es,
            "mean_objects_in_scene": round(float(dc[:, 6].sum()) / es, 3),
            "episodes_ended": int(dc[:, 7].sum()),
            "mean_contacts_per_substep": round(float(dc[:, 4].sum()) / (es * frame_skip), 3),
            "max_contacts_in_a_substep": int(dc[:, 5].max()) if len(dc) else 0,  # since creation (pre-roll incl.)
            "contacts_dropped": int(dc[:, 0].sum()),
            "newton_iters_per_substep": round(float(dc[:, 1].sum()) / (es * frame_skip), 3),
            "newton_maxiter_hits": int(dc[:, 2].sum())}


def load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


WATCHDOG_RC = 3  # exit code of a job the watchdog stopped


def stop_ranks(procs, grace=10.0):
    """SIGTERM every live rank, SIGKILL whatever is still alive after `grace` seconds"""
    for p in procs:
        if p.poll() is None:
            p.terminate()
    t0 = time.monotonic()
    while any(p.poll() is None for p in procs) and time.monotonic() - t0 < grace:
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.kill()
            p.wait()


def spawn_ranks(n, argv, deadline):
    """`bench.py --gpus N` without a torchrun environment: N rank processes of this script, one GPU each, 127.0.0.1
    rendezvous.  The parent never touches the GPU (it only waits), so nothing is exec'd from a GPU process; rank 0
    prints the JSON line.  Returns the first non-zero rank exit code (the other ranks are then stopped).
    Watchdog: a job still running `deadline` seconds after launch (a rank stuck in a collective holds every other
    rank in it) is stopped -- every rank terminated, the ranks that had not finished named on stderr -- and the
    parent exits with WATCHDOG_RC."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    pending = list(range(n))
    t0 = time.monotonic()
    while pending:
        for r in list(pending):
            code = procs[r].poll()
            if code is None:
                continue
            pending.remove(r)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench.py: rank {r} exited with {code}; stopping ranks {pending}", file=sys.stderr, flush=True)
                stop_ranks([procs[q] for q in pending])
        if pending and deadline > 0 and time.monotonic() - t0 > deadline:
            print(json.dumps({"error": "watchdog", "deadline_s": deadline, "ranks_unfinished": pending,
                              "ranks_finished": [r for r in range(n) if r not in pending]}), file=sys.stderr, flush=True)
            stop_ranks([procs[q] for q in pending])
            return WATCHDOG_RC
        time.sleep(0.2)
    return rc


def resolve_world(args):
    """None = run in this process; otherwise the exit code of the spawned ranks"""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            return spawn_ranks(args.gpus, sys.argv[1:], args.deadline)
        args.gpus = 1
        return None
    w = int(env_world)
    if args.gpus is None:
        args.gpus = w
    if args.gpus != w:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={w}")
    return None


def main_dry_run(args):
    """the launch path without a GPU (tests/test_distributed.py): gloo ranks, the arena partition and the
    max-over-ranks clock of the real run, a synthetic wall time per rank"""
    import torch.distributed as dist

    ctx = RankContext.from_env(use_gpu=False)
    lo, hi = rank_arenas(args.arenas, ctx.world, ctx.rank, args.scaling)
    if args.stall_rank == ctx.rank:
        time.sleep(args.stall_seconds)  # watchdog test: this rank arrives late at the collectives below
    ranges = [None] * ctx.world
    if ctx.distributed:
        dist.all_gather_object(ranges, (lo, hi))
    else:
        ranges = [(lo, hi)]
    per_rank = ctx.gather_rank_times(1.0 + 0.5 * ctx.rank, 0.0)
    wall = ctx.max_over_ranks(1.0 + 0.5 * ctx.rank)
    total = ctx.sum_over_ranks(hi - lo)
    if ctx.rank == 0:
        print(json.dumps({"metric": "dry run (launcher only)", "n_gpus": ctx.world, "scaling": args.scaling,
                          "backend": ctx.backend, "rank_arenas": [list(r) for r in ranges], "total_arenas": int(total),
                          "wall_max": wall, "value": total * args.steps / wall, "per_rank": per_rank}), flush=True)
    ctx.close()


def job_arenas(args, world):
    """arenas stepped by the whole job"""
    return args.arenas * world if args.scaling == "weak" else args.arenas


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default WORLD_SIZE or 1")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --arenas per GPU; strong: --arenas for the whole job, split over the ranks")
    ap.add_argument("--dry-run", action="store_true", help="launcher / partition only, no GPU (tests)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--arenas", type=int, default=4096, help="arenas per GPU")
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=4)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--preroll", type=int, default=200, help="env-steps of desynchronising pre-roll")
    ap.add_argument("--seeds", default="fixed", choices=["fixed", "arena"],
                    help="scene/TaskManager seed: 42 everywhere (saved runs) or 42 + global arena id")
    ap.add_argument("--fp64-steps", type=int, default=30, help="also time the fp64 build (0 = skip)")
    ap.add_argument("--solver-tolerance", type=float, default=0.0,
                    help="Newton tolerance (0 = the precision's default, fm_create)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 --pmc (tools/pmc_traffic.py)")
    ap.add_argument("--valu-json", default=os.path.join(ROOT, "profiles", "pmc_valu.json"),
                    help="VALU instruction counts per arena env-step by rocprofv3 --pmc (tools/pmc_valu.py)")
    ap.add_argument("--workload", default="config2", choices=["config2", "config3", "config4", "config5"],
                    help="config2: the headline (random policy); config3: 16384 arenas 2x8 PPO rollout; config4: "
                         "131072 arenas 2x8 PPO rollout strong-split over the ranks (RCCL update); config5: "
                         "4 arms x 16 objects PauseIKToggleEnv, 4096 arenas per GPU (32768 on 8), random toggles")
    ap.add_argument("--deadline", type=float, default=1200.0,
                    help="--gpus N launcher: stop every rank and exit non-zero after this many seconds (0 = none)")
    ap.add_argument("--stall-rank", type=int, default=-1, help=argparse.SUPPRESS)  # watchdog test (--dry-run)
    ap.add_argument("--stall-seconds", type=float, default=0.0, help=argparse.SUPPRESS)
    ap.add_argument("--ppo-batch", type=int, default=16384)
    ap.add_argument("--ppo-epochs", type=int, default=10)
    args = ap.parse_args()
    args.env_class = "AllFullRLProgressRewardEnv"
    if args.workload == "config4":
        if args.arenas == 4096:
            args.arenas = 131072
        args.scaling = "strong"
    rc = resolve_world(args)
    if rc is not None:
        return rc
    if args.dry_run:
        return main_dry_run(args)
    if args.workload in ("config3", "config4"):
        return main_config3(args)
    if args.workload == "config5":
        return main_config5(args)

    ctx = RankContext.from_env()
    A, K = args.arms, args.objects
    lo, hi = rank_arenas(args.arenas, ctx.world, ctx.rank, args.scaling)
    N = hi - lo  # this rank's arenas
    NJ = job_arenas(args, ctx.world)
    wall, kern_ms, dc = timed_run(ctx, args, args.precision, args.steps, args.warmup, lo, hi)
    per_rank = ctx.gather_rank_times(wall, kern_ms)
    wall = ctx.max_over_ranks(wall)
    value = NJ * args.steps / wall
    diag = diagnostics(dc, N, args.steps)
    fp64 = None
    if args.fp64_steps > 0 and args.precision == "fp32":
        w64, k64, dc64 = timed_run(ctx, args, "fp64", args.fp64_steps, min(args.warmup, 5), lo, hi)
        w64 = ctx.max_over_ranks(w64)
        fp64 = {"value": round(NJ * args.fp64_steps / w64, 2), "steps": args.fp64_steps,
                "ms_per_step": round(w64 / args.fp64_steps * 1e3, 4), "kernel_ms_avg": round(k64, 4),
                "diagnostics": diagnostics(dc64, N, args.fp64_steps)}
    if ctx.rank == 0:
        roof = make_roofline(args, N, A, K, kern_ms, args.traffic_json, args.valu_json, wall / args.steps * 1e3)
        line = {
            "metric": "env-steps/sec (whole node), 4096 arenas 2-arm×4-obj; 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "env-steps/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "f64",
            "data": f"synthetic (random U[-1,1] AllFullRL actions, Philox seed 0+rank; scene seed "
                    f"{'42' if args.seeds == 'fixed' else '42+arena id'}; {args.preroll}-step desynchronising pre-roll)",
            "config": {"workload": f"config 2: {N} arenas/GPU, {A} arms x {K} objects, AllFullRLProgressRewardEnv, "
                                   "random policy, 100 substeps/env-step, auto-reset, stationary episode mix",
                       "arenas_per_gpu": N, "job_arenas": NJ, "num_arms": A, "max_num_objects": K,
                       "parallelism": f"arena-sharded x{ctx.world} (no collective)"},
            "roofline": roof,
            "diagnostics": diag,
        }
        if ctx.world > 1:
            line["per_rank"] = per_rank
        if fp64 is not None:
            line["fp64_value"] = fp64
        if ctx.world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(A, K, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    ctx.close()


def make_roofline(args, N, A, K, kern_ms, traffic_json, valu_json, step_ms=None):
    """the line's roofline block for the dominant kernel (the env-step kernel): SURVEY §8(d)'s algorithmic bytes per
    arena env-step x the arenas of one launch / the kernel's event-timed average launch (fm_get_kernel_time), the PMC
    memory-fabric traffic per launch and the VALU work (profiles/, rocprofv3 passes) when they were taken on this
    workload.  `frac` is the step kernel's (its launch alone, as the contract's dominant-kernel roofline); "env_step"
    gives the same bytes over the whole timed env-step (step_ms: the dispatch-order kernel, the rerun-list reset and
    the wide rerun launch included -- and, for config 3, the policy)"""
    B = algorithmic_bytes(A, K)
    achieved = N * B / (kern_ms * 1e-3) / 1e9
    tj = load_json(traffic_json) or {}
    traffic = None
    if tj.get("arenas") == N and tj.get("precision") == args.precision and tj.get("A") == A and tj.get("K") == K:
        traffic = tj.get("hbm_bytes_per_launch")
    roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic,
            "frac_basis": "the step kernel's event-timed average launch (fm::step_kernel alone)",
            "kernel": "fm::step_kernel", "kernel_ms_avg": round(kern_ms, 4),
            "algorithmic_bytes_per_arena_step": B,
            "binding": "neither HBM nor MFMA: dependent LDS / VALU (fp32 + fp64) / L2 latency chains, one arena per "
                       "wave (config 2: two waves per SIMD)"}
    if step_ms:
        a2 = N * B / (step_ms * 1e-3) / 1e9
        roof["env_step"] = {"achieved": round(a2, 3), "frac": round(a2 / HBM_PEAK_GBPS, 6), "ms": round(step_ms, 4),
                            "basis": "wall-clock ms_per_step of the timed region (every launch of the env-step)"}
    if traffic is not None:
        roof["traffic_note"] = ("PMC TCC -> memory-fabric bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, "
                                + os.path.relpath(traffic_json, ROOT) + "): the per-arena scratch blocks (contact "
                                "records, Hessian) written back when the L2 evicts them, whether the MALL or HBM takes "
                                "them (no register spills since round 5); %.2f %% of the HBM peak at this launch time"
                                % (100.0 * traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS))
    vj = load_json(valu_json) or {}
    if vj.get("A") == A and vj.get("K") == K and vj.get("precision") == args.precision:
        flops = vj["valu_lane_flops_per_arena_step"] * N
        vinst = vj["valu_wave_instr_per_arena_step"] * N
        t = kern_ms * 1e-3
        peak = FP32_PEAK_TFLOPS if args.precision == "fp32" else FP64_PEAK_TFLOPS
        frac = flops / t / 1e12 / peak
        note = "lane FLOPs of executed fp32 VALU instructions (all 64 lanes counted)"
        if "valu_lane_flops_f64_per_arena_step" in vj and vj.get("valu_lane_flops_f64_per_arena_step", 0) > 0 \
                and args.precision == "fp32":
            # the fp32 build's float64 work (master state, narrowphase, Newton iterate) runs at half the fp32 rate:
            # the fraction is the share of the VALU peak's time the two kinds of FLOPs take together
            f32 = vj["valu_lane_flops_f32_per_arena_step"] * N
            f64 = vj["valu_lane_flops_f64_per_arena_step"] * N
            frac = (f32 / FP32_PEAK_TFLOPS + f64 / FP64_PEAK_TFLOPS) / t / 1e12
            note = ("lane FLOPs of executed fp32 + fp64 VALU instructions (all 64 lanes counted; fp64 priced at its "
                    "half rate in frac)")
        roof["valu"] = {"achieved": round(flops / t / 1e12, 4), "peak": peak, "unit": "TFLOP/s",
                        "frac": round(frac, 5),
                        "issue_frac": round(vinst * 2 / (t * 2.4e9 * 256 * 4), 5),
                        "note": note + " and VALU issue cycles (2 per wave-instruction) over the chip's SIMD-cycles at "
                                "2.4 GHz; counts per arena env-step from " + os.path.relpath(valu_json, ROOT)}
    return roof


def main_config5(args):
    """BASELINE config 5: 4 arms x 16 objects, PauseIKToggleEnv (IK base policy on every arm, MultiDiscrete toggles),
    4096 arenas per GPU; random fair-coin toggles (the IK proposals drive the arms), auto-reset"""
    args.arms, args.objects, args.env_class = 4, 16, "PauseIKToggleEnv"
    if args.steps == 100:
        args.steps = 20
    if args.warmup == 10:
        args.warmup = 2
    if args.preroll == 200:
        args.preroll = 100
    ctx = RankContext.from_env()
    A, K = args.arms, args.objects
    lo, hi = rank_arenas(args.arenas, ctx.world, ctx.rank, args.scaling)
    N = hi - lo
    wall, kern_ms, dc = timed_run(ctx, args, args.precision, args.steps, args.warmup, lo, hi)
    per_rank = ctx.gather_rank_times(wall, kern_ms)
    wall = ctx.max_over_ranks(wall)
    value = job_arenas(args, ctx.world) * args.steps / wall
    if ctx.rank == 0:
        line = {
            "metric": "env-steps/sec (whole node), 4096 arenas/GPU 4-arm x 16-obj PauseIKToggleEnv; MI355X",
            "value": round(value, 2), "unit": "env-steps/s", "n_gpus": ctx.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "f32" if args.precision == "fp32" else "f64",
            "data": f"synthetic (fair-coin MultiDiscrete toggles, Philox seed 0+rank; scene seed 42; {args.preroll}-step "
                    "desynchronising pre-roll)",
            "config": {"workload": f"config 5: {N} arenas/GPU, {A} arms x {K} objects, PauseIKToggleEnv (float64 IK "
                                   "base policy in the kernel), random toggles, 100 substeps/env-step, auto-reset",
                       "arenas_per_gpu": N, "num_arms": A, "max_num_objects": K,
                       "parallelism": f"arena-sharded x{ctx.world} (no collective)"},
            "kernel_ms_avg": round(kern_ms, 4),
            "roofline": make_roofline(args, N, A, K, kern_ms, os.path.join(ROOT, "profiles", "pmc5_traffic.json"),
                                      os.path.join(ROOT, "profiles", "pmc5_valu.json"), wall / args.steps * 1e3),
            "diagnostics": diagnostics(dc, N, args.steps),
        }
        if ctx.world > 1:
            line["per_rank"] = per_rank
        print(json.dumps(line), flush=True)
    ctx.close()


def main_config3(args):
    """BASELINE config 3: 16384 arenas, 2 arms x 8 objects, PPO rollout with the PyTorch-ROCm policy, 1 MI355X
    (per GPU with --gpus N: weak scaling, gradient / advantage all-reduce in the PPO update only).
    BASELINE config 4 (--workload config4): 131072 arenas of the same scene strong-split over the ranks
    (16384 per GPU on 8), the same PPO rollout, the update's gradient and advantage all-reduces over RCCL"""
    c4 = args.workload == "config4"
    if args.arenas == 4096:
        args.arenas = 16384
    if args.objects == 4:
        args.objects = 8
    if args.steps == 100:
        args.steps = 16
    if args.warmup == 10:
        args.warmup = 2
    ctx = RankContext.from_env()
    A, K = args.arms, args.objects
    lo, hi = rank_arenas(args.arenas, ctx.world, ctx.rank, args.scaling)
    N = hi - lo
    NJ = job_arenas(args, ctx.world)
    wall, train_s, dc, kern_ms = timed_run_ppo(ctx, args, lo, hi)
    per_rank = ctx.gather_rank_times(wall, train_s * 1e3)
    wall = ctx.max_over_ranks(wall)
    train_s = ctx.max_over_ranks(train_s)
    value = NJ * args.steps / wall
    samples = NJ * args.steps
    if ctx.rank == 0:
        name = "config 4" if c4 else "config 3"
        line = {
            "metric": (f"env-steps/sec (whole node), {NJ} arenas 2-arm×8-obj PPO rollout sharded over {ctx.world} "
                       "MI355X" if c4 else "env-steps/sec (whole node), 16384 arenas 2-arm×8-obj PPO rollout; MI355X"),
            "value": round(value, 2), "unit": "env-steps/s", "n_gpus": ctx.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "f32" if args.precision == "fp32" else "f64",
            "data": "synthetic: PPO rollout of a freshly initialised MlpPolicy [128, 128] (SB3 init), Gaussian "
                    f"sampling (per-rank stream); scene seed 42; {args.preroll}-step desynchronising pre-roll",
            "config": {"workload": f"{name}: {N} arenas/GPU ({NJ} in the job), {A} arms x {K} objects, "
                                   "AllFullRLProgressRewardEnv, PPO rollout (policy forward + sampling + env-step + "
                                   "buffer writes timed)",
                       "arenas_per_gpu": N, "job_arenas": NJ, "num_arms": A, "max_num_objects": K,
                       "parallelism": f"arena-sharded x{ctx.world}; RCCL all-reduce in the update only"},
            "ppo_update": {"seconds": round(train_s, 4), "samples": samples,
                           "samples_per_s": round(samples / train_s, 1),
                           "n_epochs": args.ppo_epochs, "batch_size_per_rank": args.ppo_batch,
                           "collectives": ("per minibatch: async all-reduce of the advantage statistics + one fused "
                                           "gradient all-reduce; per rollout: episode statistics"
                                           if ctx.world > 1 else "none (1 rank)")},
            "iteration_env_steps_per_s": round(samples / (wall + train_s), 2),
            "kernel_ms_avg": round(kern_ms, 4),
            "roofline": make_roofline(args, N, A, K, kern_ms, os.path.join(ROOT, "profiles", "pmc3_traffic.json"),
                                      os.path.join(ROOT, "profiles", "pmc3_valu.json"), wall / args.steps * 1e3),
            "diagnostics": diagnostics(dc, N, args.steps),
        }
        if ctx.world > 1:
            line["per_rank"] = per_rank  # kernel_ms = this rank's PPO update
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    sys.exit(main() or 0)
