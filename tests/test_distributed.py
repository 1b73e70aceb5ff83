"""Multi-rank launch path on CPU (gloo, world size 2): RankContext.from_env reads the torchrun environment and
opens the group, each rank owns its own arena ids (weak scaling, no data-path collective), the job time is the
slowest rank's and the throughput counts every rank's env-steps (factory_marl_amd/launch.py, bench.py)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from factory_marl_amd import launch

    ctx = launch.RankContext.from_env(use_gpu=False)
    assert ctx.backend == "gloo" and ctx.distributed
    lo, hi = launch.rank_arenas(4096, ctx.world, ctx.rank, "weak")
    slo, shi = launch.rank_arenas(131072, ctx.world, ctx.rank, "strong")
    seeds = launch.arena_seeds(lo, hi, "arena")
    wall = 1.0 + rank  # rank 1 is the slow one
    wmax = ctx.max_over_ranks(wall)
    total = ctx.sum_over_ranks(hi - lo)
    import bench

    value = bench.job_throughput(hi - lo, 10, ctx.world, wmax)
    out[rank] = (wmax, value, (lo, hi), (slo, shi), int(seeds[0]), total)
    ctx.barrier()
    ctx.close()


def test_rank_context_and_partition_gloo():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    assert res[0][0] == res[1][0] == 2.0  # max over ranks
    assert res[0][1] == pytest.approx(2 * 4096 * 10 / 2.0)
    assert res[0][2] == (0, 4096) and res[1][2] == (4096, 8192)  # weak: disjoint global arena ids
    assert res[0][3] == (0, 65536) and res[1][3] == (65536, 131072)  # config 4 split
    assert res[0][4] == 42 and res[1][4] == 42 + 4096
    assert res[0][5] == res[1][5] == 8192


def test_arena_range_covers_every_arena_once():
    from factory_marl_amd.launch import arena_range

    for total, world in [(131072, 8), (32768, 8), (10, 3), (7, 7)]:
        ids = np.concatenate([np.arange(*arena_range(total, world, r)) for r in range(world)])
        assert np.array_equal(ids, np.arange(total))
    with pytest.raises(ValueError):
        arena_range(3, 4, 0)


def test_single_rank_identity():
    import bench
    from factory_marl_amd import launch

    os.environ.pop("WORLD_SIZE", None)
    ctx = launch.RankContext.from_env(use_gpu=False)
    assert ctx.world == 1 and not ctx.distributed
    assert ctx.max_over_ranks(3.5) == 3.5
    assert bench.max_over_ranks(3.5) == 3.5
    assert bench.job_throughput(4096, 10, 1, 2.0) == pytest.approx(20480.0)


def test_bench_diagnostics_arithmetic():
    import bench

    dc = np.zeros((4, 8), np.int64)
    dc[:, 4] = 1000  # contacts over 100 substeps x 10 steps per arena
    dc[:, 5] = [3, 9, 4, 1]
    dc[:, 6] = 25
    dc[:, 7] = [0, 1, 0, 1]
    d = bench.diagnostics(dc, 4, 10)
    assert d["mean_contacts_per_substep"] == 1.0 and d["max_contacts_in_a_substep"] == 9
    assert d["mean_objects_in_scene"] == 2.5 and d["episodes_ended"] == 2
    assert bench.algorithmic_bytes(2, 4) == 120480


def _run_bench(*args):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dry-run", *args], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("scaling,ranges,total", [("weak", [[0, 4096], [4096, 8192]], 8192),
                                                  ("strong", [[0, 2048], [2048, 4096]], 4096)])
def test_bench_gpus_flag_launches_ranks(scaling, ranges, total):
    """`bench.py --gpus 2` (no torchrun environment) starts two rank processes itself: the line reports
    n_gpus 2, the ranks own disjoint arena ids (weak: 4096 each; strong: the 4096 total split), and the job
    clock is the slower rank's"""
    d = _run_bench("--gpus", "2", "--scaling", scaling, "--steps", "10")
    assert d["n_gpus"] == 2 and d["backend"] == "gloo"
    assert d["rank_arenas"] == ranges and d["total_arenas"] == total
    assert d["wall_max"] == 1.5 and d["value"] == pytest.approx(total * 10 / 1.5)


def test_bench_single_rank_and_config4_split():
    d = _run_bench("--steps", "4")
    assert d["n_gpus"] == 1 and d["rank_arenas"] == [[0, 4096]]
    d4 = _run_bench("--gpus", "2", "--workload", "config4")
    assert d4["scaling"] == "strong" and d4["rank_arenas"] == [[0, 65536], [65536, 131072]]


def test_bench_watchdog_stops_a_stalled_job():
    """`bench.py --gpus 2` with a rank that never reaches the collectives (it sleeps past the deadline): the parent
    stops every rank at the deadline, names the unfinished ranks on stderr and exits non-zero"""
    import json
    import subprocess
    import sys
    import time

    import bench

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dry-run", "--gpus", "2", "--deadline", "20",
                          "--stall-rank", "1", "--stall-seconds", "600"], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == bench.WATCHDOG_RC, (out.returncode, out.stderr[-2000:])
    assert time.monotonic() - t0 < 120
    rec = [json.loads(ln) for ln in out.stderr.splitlines() if ln.startswith('{"error"')]
    assert rec and rec[0]["error"] == "watchdog" and 1 in rec[0]["ranks_unfinished"], out.stderr[-2000:]
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]  # no result line from a stopped job


def test_bench_line_carries_per_rank_times():
    d = _run_bench("--gpus", "2", "--steps", "10")
    assert [r["rank"] for r in d["per_rank"]] == [0, 1]
    assert [r["wall_s"] for r in d["per_rank"]] == [1.0, 1.5]
