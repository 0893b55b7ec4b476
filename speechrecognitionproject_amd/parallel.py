"""Data parallelism for the train step: one process per GPU, the per-clip batch
sharded across ranks, ONE all-reduce(SUM) of the flat fp32 gradient buffer per step through
RCCL (torch.distributed backend "nccl" on ROCm = RCCL over xGMI), 1/world folded into Adam.

The reference has no distributed code; this is new work required by
north_star.  Ranks are launched by ``torch.distributed.run`` (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT in the environment).  On a CPU-only host the same code runs over gloo
(tests/test_parallel.py).
"""
import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def init_from_env(backend=None):
    """Initialise the default process group if WORLD_SIZE > 1; returns (rank, world, local_rank)."""
    world, rank, local = env_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        # a long timeout: rank 0 alone runs the reference's per-epoch accuracy passes while the other
        # ranks wait at a barrier (training.py)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=int(os.environ.get("SRK_DIST_TIMEOUT", "7200"))))
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def barrier():
    if world_size() > 1:
        dist.barrier()


def broadcast_flat(flat):
    """Make every rank start from rank 0's parameters (one broadcast of the flat buffer)."""
    if world_size() > 1:
        dist.broadcast(flat.data, src=0)


def allreduce_grads(flat):
    """Sum the flat gradient buffer over ranks (one collective per step).  The optimizer applies
    1/world through its grad_scale, so no separate scaling pass runs."""
    if world_size() > 1:
        dist.all_reduce(flat.grad, op=dist.ReduceOp.SUM)


def shard_indices(n_items, rank, world, seed, epoch=0):
    """DistributedSampler-equivalent: a seeded permutation, rank r takes every world-th item
    starting at r (padded by wrap-around so every rank gets the same count)."""
    g = torch.Generator().manual_seed(seed + epoch)
    perm = torch.randperm(n_items, generator=g)
    per = (n_items + world - 1) // world
    total = per * world
    if total > n_items:
        perm = torch.cat([perm, perm[: total - n_items]])
    return perm[rank:total:world]
