"""World-size-2 gloo run of bench.py's multi-rank logic (one sequence per rank, barrier around
the timed region, MAX-over-ranks time, SUM of frames) -- CPU only."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from multimot_track_amd import shard
    r, w, lr = shard.rank_env()
    dist.init_process_group("gloo", init_method="env://")
    dev = torch.device("cpu")
    shard.barrier(w, dev)
    elapsed = 1.5 + rank            # pretend rank r took 1.5 + r seconds
    frames = 32 * (rank + 1)
    t = shard.max_over_ranks(elapsed, w, dev)
    f = shard.sum_over_ranks(frames, w, dev)
    out[rank] = (r, w, lr, shard.sequence_seed(1003, r), t, f)
    dist.destroy_process_group()


def test_two_rank_sharding():
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(out)
    assert {res[r][0] for r in range(2)} == {0, 1}
    assert all(res[r][1] == 2 for r in range(2))
    assert res[0][3] != res[1][3]                       # independent sequences
    assert all(res[r][4] == pytest.approx(2.5) for r in range(2))   # max over ranks
    assert all(res[r][5] == pytest.approx(96.0) for r in range(2))  # all frames
