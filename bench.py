"""bench.py -- driver benchmark contract (one JSON line on rank 0).

Workload (BASELINE.json configs[2]): KITTI-03 geometry 1242x375, 2000 ORB
features, ego + 3 object motions.  Synthetic seeded street sequence (multimot_track_amd/scene.py:
ray-cast ground, facades and three moving boxes with exact depth, flow and semantic labels),
rendered straight into HBM before the timed region.  One sequence per GPU (seed 1003 + rank) by
default; --seqs-per-gpu K tracks K independent sequences per GPU (one context, stream set and
host thread each; SURVEY 8(e) allows several sequences per device), seeds 1003 + rank * K + k.

A "step" = System::TrackRGBD over one chunk of `--chunk` consecutive frames of the sequence:
batched ORB extraction for the chunk, then per frame the association (B1-B9), the ego flow solve
(PoseOptimizationFlow2Cam), object grouping, per-object PnP-RANSAC + PoseOptimizationFlow2 --
everything the reference does per frame on this path (mmt_track_rgbd_chunk_device).  Frames are
processed in order, so the tracker state carries across steps exactly as in rgbd_mmt.

Multi-GPU: one process per GPU (torchrun), independent sequences, no data-path collective;
barrier + device sync bracket the timed region; time = MAX over ranks; value = frames of all
ranks / that time ("scaling": "weak").

roofline: the batched ORB window -- k_gray_depth (A1 + A2) and the ORB launch sequence (A3-A9) --
with SURVEY 8(d)'s B_orb = 3WH + 4P + 60N plus A2's 6WH algorithmic bytes per frame x frames per
launch, over its average duration from HIP events the library records on the launch stream around
every window (mmt_profile_*), vs the 8 TB/s HBM peak.
cpu_baseline: the CPU oracle tracker (oracle/track_ref.cpp, a scalar C++ restatement of the
reference's per-frame path) on rank 0 over the first frames of the same sequence, 1 core.
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
METRIC = "KITTI RGB-D frames/sec (ego+object poses) at 1/2/4/8 GPUs; CPU ref fps"


def b_orb(w, h, nfeat, lw, lh):
    """Algorithmic bytes per frame of the profiled ORB window: SURVEY 8(d)'s B_orb = 3WH (BGR
    read, A1) + 4P (pyramid write + read, blurred write + read) + 60N (keypoints + descriptors),
    plus 6WH for A2, which the same fused kernel does (u16 disparity in, f32 depth out)."""
    P = int(sum(int(a) * int(b) for a, b in zip(lw, lh)))
    return 3 * w * h + 4 * P + 60 * nfeat + 6 * w * h


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for the CPU baseline record."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def load_traffic(path, cfg_key):
    """HBM bytes per ORB launch sequence from a committed rocprofv3 --pmc summary (or None)."""
    try:
        d = json.load(open(path))
        return d.get(cfg_key)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=128,
                    help="frames per step (ORB batch; SURVEY 8(d): >= 64 frames in flight)")
    ap.add_argument("--width", type=int, default=1242)
    ap.add_argument("--height", type=int, default=375)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--objects", type=int, default=3)
    ap.add_argument("--seqs-per-gpu", type=int, default=1,
                    help="independent sequences tracked concurrently on each GPU")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import multimot_track_amd as M
    from multimot_track_amd import scene, shard

    rank, world, local = shard.rank_env()
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    W, H, NF, C, K = args.width, args.height, args.nfeatures, args.chunk, args.seqs_per_gpu
    nframes = (args.warmup + args.steps) * C
    t_gen = time.perf_counter()
    def render(seed):
        # in pieces of 400 frames (each frame is rendered on its own, so the sequence is the
        # same), with a progress line on stderr for long runs under a profiler
        parts = []
        for s0 in range(0, nframes, 400):
            parts.append(scene.kitti_like_sequence(min(400, nframes - s0), W, H,
                                                   n_objects=args.objects, seed=seed,
                                                   device=dev, start=s0))
            print("rank %d: rendered %d / %d frames" % (rank, s0 + len(parts[-1]["Tcw"]),
                                                         nframes), file=sys.stderr, flush=True)
        out = {k: torch.cat([p[k] for p in parts]) for k in ("bgr", "disp", "flow", "mask")}
        out["Tcw"] = np.concatenate([p["Tcw"] for p in parts])
        return out

    seqs = [render(shard.sequence_seed(1003, rank * K + k)) for k in range(K)]
    seq = seqs[0]
    torch.cuda.synchronize(dev)
    t_gen = time.perf_counter() - t_gen

    cfg = M.kitti03_config(W, H, NF, max_batch=C, device_id=local)
    ctxs = [M.Context(cfg) for _ in range(K)]
    ctx = ctxs[0]
    lv = ctx.levels()
    # dedicated (non-default) streams: the library launches on them and records its HIP events
    # on them; torch.cuda.synchronize below waits for all of them
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    torch.cuda.set_stream(streams[0])

    def step_k(k, i):
        sl = slice(i * C, (i + 1) * C)
        s = seqs[k]
        return ctxs[k].track_chunk_device(s["bgr"][sl], s["disp"][sl], s["flow"][sl],
                                          s["mask"][sl], streams[k].cuda_stream, parse=False)

    pool = None
    if K > 1:  # one host thread per sequence (the C-ABI calls release the GIL)
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=K)

    def step(i):
        if pool is None:
            return step_k(0, i)
        return [f.result() for f in [pool.submit(step_k, k, i) for k in range(K)]][0]

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    ctx.profile_enable(True)
    ctx.profile_read(reset=True)
    shard.barrier(world, dev)
    t0 = time.perf_counter()
    results = [step(args.warmup + i) for i in range(args.steps)]
    torch.cuda.synchronize(dev)
    shard.barrier(world, dev)
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    elapsed = shard.max_over_ranks(elapsed, world, dev)
    frames_all = shard.sum_over_ranks(args.steps * C * K, world, dev)

    # per-frame outputs of the timed region (sanity: every frame tracked, objects found)
    res, objs = results[-1]
    n_obj_last = int(res[C - 1].n_objects)
    tracked = sum(int(r.initialized) for rr, _ in results for r in rr)
    gt = seq["Tcw"][-1]
    ego_err = float(np.abs(np.array(res[C - 1].Tcw[:]).reshape(4, 4) - gt).max())

    if rank == 0:
        value = frames_all / elapsed
        launch_ms = prof["orb_ms"] / max(prof["orb_launches"], 1)
        bytes_per_launch = C * b_orb(W, H, NF, lv["level_w"], lv["level_h"])
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        key = "%dx%d_n%d_b%d" % (W, H, NF, C)
        traffic = load_traffic(args.traffic_file, key)
        cpu = None
        if not args.no_cpu:
            from oracle import oracle as O
            O.build()
            kcam = (cfg.fx, cfg.fy, cfg.cx, cfg.cy)
            tr = O.Tracker(W, H, kcam, cfg.bf, 0, NF)
            n_done, tcpu = 0, 0.0
            # one pinned core (the process's first allowed CPU), restored afterwards
            affinity = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
            if affinity:
                os.sched_setaffinity(0, {min(affinity)})
            try:
                while tcpu < args.cpu_seconds and n_done < nframes:
                    f = scene.to_numpy_frames({k: seq[k][n_done:n_done + 1]
                                               for k in ("bgr", "disp", "flow", "mask")})[0]
                    tc = time.perf_counter()
                    tr.track(f["bgr"], f["disp"], f["flow"], f["sem"])
                    tcpu += time.perf_counter() - tc
                    n_done += 1
            finally:
                if affinity:
                    os.sched_setaffinity(0, affinity)
            cpu = {"value": round(n_done / tcpu, 3), "unit": "frames/s", "cores": 1,
                   "kind": "port", "cpu_model": cpu_model(), "nproc": os.cpu_count(),
                   "sample": "first %d frames of the same C3 sequence, full per-frame tracking "
                             "(oracle/track_ref.cpp: ORB, association, ego + object solves), "
                             "single thread pinned to one core, %.1f s of CPU time"
                             % (n_done, tcpu)}
        out = {
            "metric": METRIC,
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic (seeded ray-cast street sequence, exact depth/flow/"
                                   "labels, KITTI-03 camera), resident in HBM",
            "config": {"workload": "C3: KITTI-03-like RGB-D, end-to-end TrackRGBD (ORB + "
                                   "association + ego + %d object motions)" % args.objects,
                       "width": W, "height": H, "orb_features": NF, "chunk_frames": C,
                       "sequences_per_gpu": K, "parallelism": "dp%d" % world,
                       "frames_tracked": tracked, "objects_last_frame": n_obj_last,
                       "ego_abs_err_last_frame": round(ego_err, 5),
                       "scene_render_s": round(t_gen, 2)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "kernel": "batched ORB window (k_gray_depth, k_resize, k_fast, "
                                   "k_octree, k_blur, k_orient_desc) over %d frames" % C,
                         "launch_ms": round(launch_ms, 4), "bytes_per_launch": bytes_per_launch,
                         "orb_share_of_step": round(prof["orb_ms"] / (elapsed * 1e3), 4)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    if pool is not None:
        pool.shutdown()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
