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


# BASELINE.json configs: the per-rank workload of bench.py --config.
# C4: KITTI 00 / 03 / 05 / 07 geometries and lengths, one sequence per rank (rank r -> entry
# r mod 4), 4000 features, ego + 3 moving boxes, seed 1000 + sequence number.  C5: 1920x1080,
# 8000 features, two boxes each split into four rigid column bands with labels of their own
# (eight rigid object motions; the reference's loader keeps labels 1..3 only, rgbd_tum.cc:335, so
# eight motions need that filter lifted: SURVEY's documented deviation), seed 2000 + rank.
C4_SEQUENCES = (("00", 1241, 376, 4541), ("03", 1242, 375, 801), ("05", 1226, 370, 2761),
                ("07", 1226, 370, 1101))
C5_LANES = [(-3.0, 12.0), (3.4, 9.0)]


def workload(config, rank):
    """dict(name, width, height, nfeatures, objects, lanes, parts, length, seed) of `rank`."""
    if config == "C2":
        return dict(name="C2", width=1242, height=375, nfeatures=2000, objects=0, lanes=None,
                    parts=1, length=None, seed=sequence_seed(1003, rank))
    if config == "C3":
        return dict(name="C3", width=1242, height=375, nfeatures=2000, objects=3, lanes=None,
                    parts=1, length=None, seed=sequence_seed(1003, rank))
    if config == "C4":
        sq, w, h, n = C4_SEQUENCES[rank % len(C4_SEQUENCES)]
        return dict(name="C4/KITTI-%s" % sq, width=w, height=h, nfeatures=4000, objects=3,
                    lanes=None, parts=1, length=n, seed=1000 + int(sq))
    if config == "C5":
        return dict(name="C5", width=1920, height=1080, nfeatures=8000, objects=2,
                    lanes=C5_LANES, parts=4, length=None, seed=sequence_seed(2000, rank))
    raise ValueError("unknown config %r" % config)


def rank_steps(length, chunk, warmup, steps):
    """(warmup, timed) steps of a rank whose sequence holds `length` frames (None: unbounded):
    a shorter sequence times fewer chunks (the others' time still bounds the job: MAX over
    ranks, frames summed)."""
    if length is None:
        return warmup, steps
    n = length // chunk
    w = min(warmup, n)
    return w, max(0, min(steps, n - w))
