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


def test_bench_self_launches_ranks_dry():
    """bench.py --gpus 2 outside torchrun starts its own two ranks (torch.distributed.run child,
    gloo in --dry mode) and reports the world size the process group was initialised with, the
    per-rank sequence seeds, MAX-over-ranks time and the frames of all ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry",
                        "--steps", "3", "--warmup", "1", "--chunk", "8"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["seeds"] == [[1003], [1004]]
    assert d["config"]["frames_all"] == 2 * 3 * 8
    # the slower rank (2 x 10 ms per step) sets the time: 3 steps >= 60 ms
    assert d["ms_per_step"] >= 20.0
    assert d["value"] == pytest.approx(48 / (d["ms_per_step"] * 3 / 1000.0), rel=0.02)


def test_bench_c4_per_rank_workloads_dry():
    """bench.py --config C4: rank r tracks KITTI 00 / 03 / 05 / 07's geometry, length and seed
    (shard.workload); a rank whose sequence ends early times fewer chunks, the job's time is still
    the MAX over ranks and its frames the SUM of what every rank timed (dry gloo rehearsal with
    the lengths scaled down so that rank 1's KITTI-03 runs out)."""
    import json
    import subprocess
    import sys
    from multimot_track_amd import shard
    assert [shard.workload("C4", r)["name"] for r in range(4)] == \
        ["C4/KITTI-00", "C4/KITTI-03", "C4/KITTI-05", "C4/KITTI-07"]
    assert (shard.workload("C4", 2)["width"], shard.workload("C4", 2)["height"]) == (1226, 370)
    assert shard.workload("C5", 3)["nfeatures"] == 8000 and shard.workload("C5", 3)["parts"] == 4
    assert shard.rank_steps(801, 128, 5, 20) == (5, 1)
    assert shard.rank_steps(None, 128, 5, 20) == (5, 20)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry",
                        "--config", "C4", "--steps", "3", "--warmup", "1", "--chunk", "8",
                        "--dry-length-scale", "0.02"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    ranks = d["config"]["ranks"]
    assert [r[0]["name"] for r in ranks] == ["C4/KITTI-00", "C4/KITTI-03"]
    assert d["config"]["seeds"] == [[1000], [1003]]
    # KITTI-00 (90 frames after scaling): 1 warm-up + 3 timed chunks; KITTI-03 (16): 1 + 1
    assert [r[0]["timed_steps"] for r in ranks] == [3, 1]
    assert d["config"]["frames_all"] == (3 + 1) * 8
    # MAX over ranks: rank 0's three 10 ms steps, not rank 1's single 20 ms step
    assert d["ms_per_step"] * 3 >= 30.0


def test_bench_ranks_per_gpu_dry():
    """bench.py --ranks-per-gpu 2 on one GPU: two processes (gloo), each with its own sequence;
    n_gpus stays 1, the time is the MAX over the ranks and the frames their SUM."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--ranks-per-gpu", "2",
                        "--dry", "--steps", "3", "--warmup", "1", "--chunk", "8"], cwd=root,
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["config"]["sequences_per_gpu"] == 2
    assert d["config"]["seeds"] == [[1003], [1004]]
    assert d["config"]["frames_all"] == 2 * 3 * 8
    assert d["ms_per_step"] >= 20.0
