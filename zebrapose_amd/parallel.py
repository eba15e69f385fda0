"""Process-group plumbing for the data-parallel path (one process per GPU; backend 'nccl' is RCCL
over xGMI on ROCm, 'gloo' for CPU tests).

Reference: train_v6.py:47-51 (init_process_group), :82-91 (lr x world, iterations / world),
:149/168/223 (DistributedSampler), :391-393 (metric all-reduce of [value, 1]).
Inference shards crops by rank with no collective; training all-reduces gradients through DDP.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist


def init_from_env(backend="nccl"):
    """torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT); returns (rank, world, local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def sampler_indices(n, rank, world, epoch=0, shuffle=True, seed=0):
    """torch DistributedSampler semantics (drop_last=False): pad by wrapping to a multiple of
    world, then every world-th index starting at rank."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    total = int(math.ceil(n / world)) * world
    idx += idx[: total - len(idx)]
    return idx[rank:total:world]


def crop_shard(n, rank, world):
    """Contiguous crop range [lo, hi) of rank for inference (no collective needed)."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def all_reduce_mean_metric(value, device=None):
    """train_v6.py:391-393: all_reduce SUM of [value, 1] -> value / count."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value), 1.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return (t[0] / t[1]).item()


def max_over_ranks(seconds, device=None):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()
