"""One process per GPU: rank context, arena partition and job timing for the arena-sharded env-step.

Replaces the reference's only parallelism, ``make_vec_env(..., n_envs=8, vec_env_cls=SubprocVecEnv)``
(/root/reference/src/learning.py:98-100), which forks one CPU worker per environment.  Here each rank owns
one ``FactoryVecEnv`` (one HIP stream, its arenas resident in its GPU's HBM) and arenas never exchange
data, so the env-step has no collective at all.  Collectives exist only for job
timing (max over ranks) and, in the trainer, for the PPO gradient / advantage statistics.

Launch (torchrun, one rank per GPU, 127.0.0.1 rendezvous):
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N
``RankContext.from_env`` reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and opens the process group
(RCCL = backend "nccl" on ROCm for GPU ranks, gloo for CPU tests).  Nothing here touches the GPU before
``init`` picks the device, and nothing re-execs the process.
"""
import os
from dataclasses import dataclass


@dataclass
class RankContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: object = None

    @classmethod
    def from_env(cls, backend=None, use_gpu=True):
        """read the torchrun environment; open the process group when world > 1"""
        import torch

        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        ctx = cls(rank=rank, world=world, local_rank=local_rank)
        if use_gpu:
            torch.cuda.set_device(local_rank)
            ctx.device = torch.device("cuda", local_rank)
        else:
            ctx.device = torch.device("cpu")
        if world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            ctx.backend = backend or ("nccl" if use_gpu else "gloo")
            if not dist.is_initialized():
                kw = dict(device_id=ctx.device) if ctx.backend == "nccl" else {}
                dist.init_process_group(ctx.backend, rank=rank, world_size=world, **kw)
        return ctx

    @property
    def distributed(self):
        import torch.distributed as dist

        return self.world > 1 and dist.is_available() and dist.is_initialized()

    def barrier(self):
        import torch

        if self.distributed:
            import torch.distributed as dist

            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def max_over_ranks(self, x):
        return max_over_ranks(x, self.device if self.backend == "nccl" else None)

    def sum_over_ranks(self, x):
        return reduce_over_ranks(x, "sum", self.device if self.backend == "nccl" else None)

    def gather_rank_times(self, wall, kernel_ms):
        """every rank's own timed-region wall time and average kernel time, gathered to every rank (per-rank
        imbalance in an N-GPU line); a one-element list at N=1"""
        mine = {"rank": self.rank, "wall_s": round(float(wall), 4), "kernel_ms": round(float(kernel_ms), 4)}
        if not self.distributed:
            return [mine]
        import torch.distributed as dist

        out = [None] * self.world
        dist.all_gather_object(out, mine)
        return out

    def close(self):
        if self.distributed:
            import torch.distributed as dist

            dist.destroy_process_group()


def arena_range(total_arenas, world, rank):
    """contiguous arena ids [lo, hi) of `rank` when `total_arenas` are split over `world` ranks (the first
    total % world ranks take one extra arena); SURVEY.md §8(e): ids [g*N/8, (g+1)*N/8) per GPU"""
    if total_arenas < world:
        raise ValueError(f"{total_arenas} arenas cannot be split over {world} ranks")
    base, extra = divmod(total_arenas, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def rank_arenas(arenas_per_rank, world, rank, scaling="weak"):
    """arena ids of this rank: weak scaling gives every rank `arenas_per_rank` arenas (global ids
    rank*n .. rank*n + n - 1); strong scaling splits `arenas_per_rank` (then the job total) over the ranks"""
    if scaling == "weak":
        return rank * arenas_per_rank, (rank + 1) * arenas_per_rank
    if scaling == "strong":
        return arena_range(arenas_per_rank, world, rank)
    raise ValueError(scaling)


def arena_seeds(lo, hi, mode="fixed", seed=42):
    """per-arena seeds for build_scene / TaskManager (base_env.py:300, task_utils.py:19): "fixed" = the
    saved runs' seed in every arena (runs/*.json env_kwargs.seed), "arena" = seed + global arena id"""
    import numpy as np

    if mode == "fixed":
        return np.full(hi - lo, seed, np.uint64)
    if mode == "arena":
        return (seed + np.arange(lo, hi)).astype(np.uint64)
    raise ValueError(mode)


def max_over_ranks(x, device=None):
    """max of a host float over all ranks (the slowest rank's clock sets the job time); identity at N=1"""
    return reduce_over_ranks(x, "max", device)


def reduce_over_ranks(x, op="max", device=None):
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def job_throughput(arenas_per_rank, steps, world, wall_max):
    """whole-job env-steps/s: every rank steps its own arenas (weak scaling, no data-path collective)"""
    return world * arenas_per_rank * steps / wall_max
