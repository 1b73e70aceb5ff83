"""Multi-GPU bench path on CPU (gloo, world size 2): each rank times its own shard of arenas, the job time
is the slowest rank's, and the throughput counts every rank's env-steps (weak scaling, no data-path
collective)."""
import os
import socket

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
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    wall = 1.0 + rank  # rank 1 is the slow one
    wmax = bench.max_over_ranks(wall)
    value = bench.job_throughput(4096, 10, world, wmax)
    out[rank] = (wmax, value)
    dist.barrier()
    dist.destroy_process_group()


def test_max_over_ranks_and_job_throughput_gloo():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    assert res[0] == res[1]
    wmax, value = res[0]
    assert wmax == 2.0
    assert value == pytest.approx(2 * 4096 * 10 / 2.0)


def test_single_rank_identity():
    import bench

    assert bench.max_over_ranks(3.5) == 3.5
    assert bench.job_throughput(4096, 10, 1, 2.0) == pytest.approx(20480.0)
