"""bench.py -- driver benchmark contract (one JSON line on rank 0).

Workload (BASELINE.json configs[1]): KITTI-03 geometry 1242x375, 2000 ORB
features, synthetic seeded frames (value noise, scene seed 1003) resident in HBM before the timed
region.  A "step" = one pass of the hot path over one batch of `--batch` frames of one sequence.

Stage measured in this version: batched ORB extraction (ORBextractor::operator() for every frame
of the batch: pyramid, FAST cells, octree, orientation, blur, BRIEF).  config.workload names the
stage; the tracker stages are added to the timed region as they land.

Multi-GPU: one process per GPU (torchrun); each rank owns an independent sequence (different seed),
no data-path collective; barrier + cuda sync bracket the timed region; the time is the MAX over
ranks; value = frames of all ranks / that time ("scaling": "weak").

roofline: algorithmic bytes per ORB launch sequence (B_orb = 3WH + 4P + 60N per frame)
/ its average duration from HIP events on the launch stream, vs the 8 TB/s HBM peak.
cpu_baseline: the CPU oracle (oracle/, a scalar C++ restatement of the reference) on rank 0, on a
bounded sample of the same frames, 1 core.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def b_orb(w, h, nfeat, lw, lh):
    P = int(sum(int(a) * int(b) for a, b in zip(lw, lh)))
    return 3 * w * h + 4 * P + 60 * nfeat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--width", type=int, default=1242)
    ap.add_argument("--height", type=int, default=375)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import multimot_track_amd as M
    from multimot_track_amd import synthetic

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    W, H, NF, B = args.width, args.height, args.nfeatures, args.batch
    cfg = M.kitti03_config(W, H, NF, max_batch=B, device_id=local)
    ctx = M.Context(cfg)
    cap = ctx.capacity()
    lv = ctx.levels()

    # synthetic sequence of this rank (seed 1003 + rank), resident in HBM
    seed0 = 1003 + 1000 * rank
    frames = np.stack([synthetic.gray_frame(H, W, seed0 + i) for i in range(B)])
    d_gray = torch.from_numpy(frames).to(dev)
    d_kps = torch.empty((B, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.empty(B, dtype=torch.int32, device=dev)
    # a dedicated (non-default) stream: the library launches on it and the HIP events below are
    # recorded on it, so they bracket exactly the kernels of the step
    stream = torch.cuda.Stream(dev)

    def step():
        rc = M.lib().mmt_orb_extract_device(ctx.handle, d_gray.data_ptr(), B, W * H,
                                            d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                            d_n.data_ptr(), stream.cuda_stream)
        if rc != 0:
            raise M.MmtError(M.lib().mmt_last_error(ctx.handle).decode())

    torch.cuda.set_stream(stream)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    nkp = d_n.cpu().numpy()

    if rank == 0:
        frames_total = args.steps * B * world
        value = frames_total / elapsed
        bytes_per_launch = B * b_orb(W, H, NF, lv["level_w"], lv["level_h"])
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        cpu = None
        if not args.no_cpu:
            from oracle import oracle as O
            O.build()
            n_done, tc0 = 0, time.perf_counter()
            while time.perf_counter() - tc0 < args.cpu_seconds:
                O.orb_extract(frames[n_done % B], NF)
                n_done += 1
            tcpu = time.perf_counter() - tc0
            cpu = {"value": n_done / tcpu, "unit": "frames/s", "cores": 1, "kind": "port",
                   "sample": "%d synthetic 1242x375 frames, ORB extraction (oracle/orb_ref.cpp), "
                             "single thread, %.1f s" % (n_done, tcpu)}
        out = {
            "metric": "KITTI RGB-D frames/sec (ego+object poses) at 1/2/4/8 GPUs; CPU ref fps",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic (seeded value-noise frames, KITTI-03 geometry)",
            "config": {"workload": "C2 front end, stage: batched ORB extraction only "
                                   "(tracker stages not yet in the timed region)",
                       "width": W, "height": H, "orb_features": NF, "batch_frames": B,
                       "keypoints_per_frame": float(nkp.mean()), "parallelism": "dp%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None,
                         "kernel": "ORB launch sequence (k_resize..k_orient_desc), %d frames" % B,
                         "launch_ms": round(launch_ms, 4), "bytes_per_launch": bytes_per_launch},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
