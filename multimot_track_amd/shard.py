"""One-sequence-per-rank sharding for bench.py: independent sequences, no
data-path collective; a barrier brackets the timed region and the time reported is the MAX over
ranks.  Backend-agnostic so the multi-rank logic is testable on CPU with gloo."""
import os

import torch
import torch.distributed as dist


def rank_env():
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def sequence_seed(base, rank):
    """Each rank tracks its own sequence (BASELINE C4/C5: seeds base + stream)."""
    return int(base) + int(rank)


def barrier(world, device=None):
    if world > 1:
        if device is not None and device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])  # RCCL: the rank's own GPU, no guessing
        else:
            dist.barrier()
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)


def max_over_ranks(value, world, device):
    """Wall time of the slowest rank (whole-job throughput = all frames / this time)."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, world, device):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
