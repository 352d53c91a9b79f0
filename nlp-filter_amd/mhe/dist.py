"""Data-parallel plumbing: independent trajectories sharded over ranks.

One process per GPU (torch.distributed over RCCL/xGMI; ``gloo`` on CPU for
tests).  Trajectories are independent, so the data path has NO collective:
  * each rank generates / owns a contiguous shard (seed = base + 1000 * rank);
  * the model constants are broadcast once from rank 0 (setup, untimed);
  * timing takes the max over ranks, throughput the sum over ranks.
"""
import os

import torch
import torch.distributed as dist


def world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def init(backend, device=None):
    ws, _, _ = world()
    if ws > 1 and not dist.is_initialized():
        if backend == "nccl" and device is not None:
            dist.init_process_group(backend, device_id=device)
        else:
            dist.init_process_group(backend)
    return ws


def shard_seed(base, rank):
    return base + 1000 * rank


def shard_range(total, ws, rank):
    """Contiguous [lo, hi) of `total` items for `rank` (strong-scaling split)."""
    q, r = divmod(total, ws)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def broadcast_(t, src=0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(t, src=src)
    return t


def max_over_ranks(x, device):
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def sum_over_ranks(x, device):
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.item()


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
