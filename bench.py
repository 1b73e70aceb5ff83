#!/usr/bin/env python3
"""Benchmark: env-steps/sec of the batched factory-manipulation env-step on MI355X.

Metric (BASELINE.json): env-steps/sec (whole node), 4096 arenas 2-arm x 4-obj, 1/2/4/8 MI355X.
Workload (BASELINE.md / SURVEY.md §8d, config 2): 4096 arenas per GPU, A=2 arms, K=4 cubes,
AllFullRLProgressRewardEnv, random policy U[-1,1]^16 drawn from a Philox stream (seed 0 + rank) before the
timed region (policy excluded), auto-reset inside the step.  One step = one env-step of every arena
(100 physics substeps + task layer).  Multi-GPU: one process per GPU, arenas are independent (weak
scaling, no data-path collective); value = all ranks' env-steps / max-over-ranks time.

Roofline: the dominant (only) kernel in the timed region is fm::step_kernel; its average launch time is
measured with HIP events on the stream it runs on.  Algorithmic bytes per arena env-step
B(A,K) = 100*8*(nq + 2nv + nu) + 4*(act_dim + obs_dim + 4) = 120,480 B at (2,4).
CPU baseline: the oracle (our C restatement of the reference algorithm, oracle/) stepped with OpenMP on
the host cores of the same box, on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def algorithmic_bytes(A, K):
    nq, nv, nu = 1 + 7 * K + 9 * A, 1 + 6 * K + 9 * A, 1 + 8 * A
    obs_dim, act_dim = 24 * A + 13 * K, 8 * A
    return 100 * 8 * (nq + 2 * nv + nu) + 4 * (act_dim + obs_dim + 4)


def max_over_ranks(x, device=None):
    """max of a host float over all ranks (the slowest rank's clock sets the job time); identity at N=1"""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_throughput(arenas_per_rank, steps, world, wall_max):
    """whole-job env-steps/s: every rank steps its own arenas (weak scaling, no data-path collective)"""
    return world * arenas_per_rank * steps / wall_max


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
            "sample": f"{cores} arenas x {steps} env-steps ({A} arms x {K} objects, random actions), "
                      f"oracle/ C restatement (fp64, OpenMP), {dt:.1f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--arenas", type=int, default=4096, help="arenas per GPU")
    ap.add_argument("--arms", type=int, default=2)
    ap.add_argument("--objects", type=int, default=4)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 --pmc (tools/pmc_traffic.py)")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)

    from factory_marl_amd import FactoryVecEnv

    A, K, N = args.arms, args.objects, args.arenas
    env = FactoryVecEnv(N, env_kwargs=dict(num_arms=A, max_num_objects=K, seed=42), device=local_rank,
                        precision=args.precision)
    env.reset()
    g = torch.Generator(device=device)
    g.manual_seed(0 + rank)
    total = args.warmup + args.steps
    acts = torch.rand(total, N, env.act_dim, device=device, generator=g, dtype=torch.float32) * 2.0 - 1.0
    for s in range(args.warmup):
        env.step_tensors(acts[s])
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    barrier()
    stream = torch.cuda.current_stream(device)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for s in range(args.warmup, total):
        env.step_tensors(acts[s])
    ev1.record(stream)
    barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # average step_kernel launch (only kernel in the region)
    wall = max_over_ranks(wall, device)
    value = job_throughput(N, args.steps, world, wall)
    ctr = env.counters()
    dropped = int(ctr[:, 0].sum())
    diag = {"contacts_dropped": dropped, "newton_iters_per_substep": round(float(ctr[:, 1].sum()) / (N * total * 100), 3),
            "newton_maxiter_hits": int(ctr[:, 2].sum()), "arenas_with_maxiter": int((ctr[:, 2] > 0).sum())}
    if rank == 0:
        B = algorithmic_bytes(A, K)
        achieved = N * B / (kern_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("arenas") == N and tj.get("precision") == args.precision and tj.get("A") == A and tj.get("K") == K:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        line = {
            "metric": "env-steps/sec (whole node), 4096 arenas 2-arm×4-obj; 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "f64",
            "data": "synthetic (random U[-1,1] AllFullRL actions, Philox seed 0+rank; scene seed 42)",
            "config": {"workload": f"config 2: {N} arenas/GPU, {A} arms x {K} objects, AllFullRLProgressRewardEnv, "
                                   "random policy, 100 substeps/env-step, auto-reset",
                       "arenas_per_gpu": N, "num_arms": A, "max_num_objects": K,
                       "parallelism": f"arena-sharded x{world} (no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic,
                         "kernel": "fm::step_kernel", "kernel_ms_avg": round(kern_ms, 4),
                         "algorithmic_bytes_per_arena_step": B},
            "diagnostics": diag,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(A, K, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
