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


def _digest(t):
    """Position-weighted checksum of a buffer's bytes (int64, on its device): two buffers
    that differ in any byte or in byte order differ here (except by a ~2^-60 collision)."""
    b = t.detach().reshape(-1).view(torch.uint8).to(torch.int64)
    w = torch.arange(b.numel(), device=b.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([(b * w).sum(), b.sum(), torch.tensor(b.numel(), device=b.device)])


def verify_broadcast(t, device, src=0):
    """After broadcast_(t): (ranks_seen, ok_ranks) by collectives, not by the environment
    -- ranks_seen = all-reduce sum of 1 over the process group, ok_ranks = the number of
    ranks whose copy of ``t`` has rank ``src``'s digest.  One process: (1, 1)."""
    d = _digest(t).to(device)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return 1, 1
    ref = d.clone()
    dist.broadcast(ref, src=src)
    cnt = torch.tensor([1.0, float(bool(torch.equal(ref, d)))], dtype=torch.float64, device=device)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    return int(cnt[0].item()), int(cnt[1].item())


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
