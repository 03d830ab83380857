"""bench.py -- driver benchmark contract (one JSON line on rank 0).

Workload (BASELINE.json configs[2]): KITTI-03 geometry 1242x375, 2000 ORB
features, ego + 3 object motions.  Synthetic seeded street sequence (multimot_track_amd/scene.py:
ray-cast ground, facades and three moving boxes with exact depth, flow and semantic labels),
rendered straight into HBM before the timed region.  One sequence per GPU (seed 1003 + rank) by
default; --seqs-per-gpu K tracks K independent sequences per GPU (one context, stream set and
host thread each; SURVEY 8(e) allows several sequences per device), seeds 1003 + rank * K + k.

A "step" = System::TrackRGBD over one chunk of `--chunk` consecutive frames of the sequence:
batched ORB extraction for the chunk, then per frame everything the reference does on this path
(mmt_track_rgbd_chunk_device), including the synchronous LocalMapping of every new keyframe
(ComputeBoW, CreateNewMapPoints, SearchInNeighbors + Fuse, local bundle adjustment, keyframe
culling) with the DBoW2 vocabulary loaded as System loads it (--vocabulary: the committed test
vocabulary; the reference's ORBvoc.txt is missing).  Frames are processed in
order, so the tracker state carries across steps exactly as in rgbd_mmt.  By default the object
results are deferred (mmt_set_deferred_objects): the object pipeline keeps running across steps
instead of draining at every chunk boundary, each frame's object motions arrive with a later
step's results, and the timed region ends with mmt_flush_objects, so every timed frame's objects
are computed inside it (--immediate: drain at every step).  `one_frame_per_call` times the
reference-shaped call pattern (one frame per mmt_track_rgbd_chunk_device call, deferred objects)
on the frames after the timed region.

Multi-GPU: one process per GPU, independent sequences, no data-path collective; barrier + device
sync bracket the timed region; time = MAX over ranks; value = frames of all ranks / that time
("scaling": "weak").  `--gpus N` without a torchrun environment launches the N ranks itself
(torch.distributed.run as a child process; this parent never touches the GPU); n_gpus is the
world size the process group was initialised with.  --ranks-per-gpu R runs R such processes per
GPU (each its own sequences, contexts and hardware queues; gloo for the barrier and reductions):
the rate of several sequences per GPU without one process's shared queues.

roofline: the batched ORB window -- k_gray_depth (A1 + A2) and the ORB launch sequence (A3-A9) --
with SURVEY 8(d)'s B_orb = 3WH + 4P + 60N plus A2's 6WH algorithmic bytes per frame x frames per
launch, over its average duration from HIP events the library records on the launch stream around
every window (mmt_profile_*), vs the 8 TB/s HBM peak.

cpu_baseline (rank 0, N = 1 only): the CPU oracle tracker (oracle/track_ref.cpp, a scalar C++
restatement of the reference's per-frame path) on one pinned core.  It tracks the same sequence
from frame 0 (the chain has to be replayed), is timed on the frame range the GPU timed region
starts with, and every frame it tracks is compared with the GPU's result for that frame (the
"parity" record).  --cpu-seqs K adds K independent sequences on K pinned cores (BASELINE C4/C5
style), and the C2 (ego-only) workload is timed beside C3 on both sides.

--dry: CPU-only rehearsal of the rank logic (gloo, no libmmt, a fixed sleep per step); used by
tests/test_dist.py.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
METRIC = "KITTI RGB-D frames/sec (ego+object poses) at 1/2/4/8 GPUs; CPU ref fps"
WORKLOADS = {
    "C2": "C2: KITTI-03-like RGB-D, ego only (%d object motions), end-to-end TrackRGBD",
    "C3": "C3: KITTI-03-like RGB-D, end-to-end TrackRGBD (ORB + association + ego + %d object "
          "motions)",
    "C4": "C4: KITTI 00/03/05/07-like RGB-D sequences, one per rank (their geometry, length and "
          "seed), 4000 features, ego + %d object motions, end-to-end TrackRGBD",
    "C5": "C5: 1920x1080 synthetic RGB-D streams, 8000 features, ego + %d rigid object motions, "
          "end-to-end TrackRGBD",
}


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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=("C2", "C3", "C4", "C5"), default="C3",
                    help="BASELINE.json workload per rank (multimot_track_amd/shard.py workload): "
                         "C3 (default) KITTI-03 + 3 objects; C4 KITTI 00/03/05/07 geometry, "
                         "length and seed per rank at 4000 features; C5 1920x1080, 8000 "
                         "features, eight rigid object motions")
    ap.add_argument("--dry-length-scale", type=float, default=1.0,
                    help="(--dry) scale of the C4 sequence lengths: rehearses ranks whose "
                         "sequences end before the timed steps do")
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
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU time of the timed oracle leg (after the run-up to the GPU's "
                         "first timed frame)")
    ap.add_argument("--cpu-seqs", type=int, default=4,
                    help="independent sequences on as many pinned cores (0: skip)")
    ap.add_argument("--cpu-seqs-seconds", type=float, default=8.0)
    ap.add_argument("--c2-steps", type=int, default=3,
                    help="timed steps of the C2 (ego-only) leg (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--immediate", action="store_true",
                    help="every step returns its frames' own object motions (drains the object "
                         "pipeline at each chunk boundary)")
    ap.add_argument("--single-frames", type=int, default=256,
                    help="frames of the one-frame-per-call leg (0: skip)")
    ap.add_argument("--vocabulary", default=os.path.join(ROOT, "tests", "golden",
                                                          "test_voc_k10l6.txt"),
                    help="DBoW2 vocabulary (text format) every context and oracle tracker loads, as "
                         "System does (System.cc:57-67): TrackReferenceKeyFrame, Relocalization and "
                         "LocalMapping's BoW steps + CreateNewMapPoints run; '' for none (the "
                         "substitutes of DESIGN.md section 2)")
    ap.add_argument("--ranks-per-gpu", type=int, default=1,
                    help="processes per GPU, each with its own sequence(s), contexts and the "
                         "HIP runtime's hardware queues (gloo for the barrier and the reductions; "
                         "n_gpus stays the GPU count)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (0: leave it; more queues measured "
                         "slower: K=8 1461 / 733 / 299 frames/s at 4 / 16 / 32)")
    ap.add_argument("--rank-parity-frames", type=int, default=192,
                    help="frames of every sequence checked against the oracle on lines with "
                         "several sequences or ranks (0: skip)")
    ap.add_argument("--dry", action="store_true", help="CPU rehearsal of the rank logic")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(args):
    """--gpus N outside a torchrun environment: start N ranks (one per GPU) with
    torch.distributed.run as a child process and return its exit code.  Nothing here touches the
    GPU, so the ranks own their devices from the start."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus * args.ranks_per_gpu), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------ per-frame result plumbing
def frames_from_raw(raw, C):
    """(MmtFrameResult[C], MmtMotion[C * MAX_OBJECTS]) -> the per-frame dicts of Context.track."""
    import multimot_track_amd as M
    res, objs = raw
    mo = M.MAX_OBJECTS
    return [M._frame_dict(res[i], objs[i * mo:(i + 1) * mo]) for i in range(C)]


def assemble(raws, C, flushed=()):
    """Per-frame dicts in frame order with each frame's own object motions: results of deferred
    calls carry the objects of an earlier frame (objects_frame), the flush the rest."""
    frames, objs = [], {}
    for raw in raws:
        for d in frames_from_raw(raw, C):
            frames.append(d)
            if d["objects_frame"] >= 0:
                objs[d["objects_frame"]] = d["objects"]
    for f, o in flushed:
        objs[f] = o
    for d in frames:
        d["objects"] = objs.get(d["frame_index"], [])
    return frames


def seq_frame_numpy(seq, i):
    """Host copy of frame i of a device-resident sequence (oracle input layout)."""
    from multimot_track_amd import scene
    return scene.to_numpy_frames({k: seq[k][i:i + 1] for k in ("bgr", "disp", "flow", "mask")})[0]


# ------------------------------------------------------------------ CPU legs (rank 0, N = 1)
def cpu_leg(args, seq, gpu_frames, timed_from, W, H, NF):
    """The oracle on one pinned core: untimed run-up over frames [0, timed_from), then timed
    frames from `timed_from` for --cpu-seconds; every tracked frame is compared with the GPU."""
    from oracle import compare, oracle as O
    O.build()
    K = (721.5377, 721.5377, 609.5593, 172.8540)
    tr = O.Tracker(W, H, K, 387.5744, 0, NF)
    if args.vocabulary:
        tr.set_vocabulary(args.vocabulary)
    affinity = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    if affinity:
        os.sched_setaffinity(0, {min(affinity)})
    ofr = []
    n_timed, t_timed = 0, 0.0
    t_run = time.perf_counter()
    try:
        i = 0
        nmax = len(gpu_frames)
        while i < nmax:
            f = seq_frame_numpy(seq, i)
            t0 = time.perf_counter()
            ofr.append(tr.track(f["bgr"], f["disp"], f["flow"], f["sem"]))
            dt = time.perf_counter() - t0
            if i >= timed_from:
                n_timed += 1
                t_timed += dt
                if t_timed >= args.cpu_seconds:
                    break
            if i % 100 == 0:
                print("cpu leg: frame %d (%.0f s)" % (i, time.perf_counter() - t_run),
                      file=sys.stderr, flush=True)
            i += 1
    finally:
        if affinity:
            os.sched_setaffinity(0, affinity)
    par = compare.parity_record(gpu_frames[:len(ofr)], ofr)
    return n_timed, t_timed, par


def cpu_multi_leg(args, render, W, H, NF, fps1):
    """--cpu-seqs K independent sequences, one oracle process pinned to each of K cores, started
    together (BASELINE.md C4/C5 "k sequences on k cores")."""
    K = args.cpu_seqs
    affinity = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    cores = affinity[:K] if len(affinity) >= K else [-1] * K
    need = int(max(fps1, 1.0) * args.cpu_seqs_seconds * 1.5) + 8
    tmp = tempfile.mkdtemp(prefix="mmt_cpuseq_")
    procs = []
    try:
        for k in range(K):
            seq = render(2003 + k, need)
            d = os.path.join(tmp, "s%d" % k)
            os.makedirs(d)
            np.save(os.path.join(d, "bgr.npy"), seq["bgr"].cpu().numpy())
            np.save(os.path.join(d, "disp.npy"), seq["disp"].cpu().numpy().view(np.uint16))
            np.save(os.path.join(d, "flow.npy"), seq["flow"].cpu().numpy())
            np.save(os.path.join(d, "mask.npy"), seq["mask"].cpu().numpy())
            del seq
        t0 = time.perf_counter()
        for k in range(K):
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "oracle.cpu_worker", os.path.join(tmp, "s%d" % k),
                 str(cores[k]), str(args.cpu_seqs_seconds), str(W), str(H), str(NF),
                 args.vocabulary or ""],
                cwd=ROOT, stdout=subprocess.PIPE, text=True))
        outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in procs]
        wall = time.perf_counter() - t0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    rate = sum(o["frames"] / o["seconds"] for o in outs if o["seconds"] > 0)
    return {"sequences": K, "cores": K, "value": round(rate, 3), "unit": "frames/s",
            "frames": [o["frames"] for o in outs], "wall_s": round(wall, 2),
            "pinned_cores": cores,
            "sample": "%d independent C3 sequences (seeds 2003..%d), one oracle process pinned to "
                      "each core, started together, %.0f s of CPU time each; value = sum of the "
                      "per-core rates" % (K, 2002 + K, args.cpu_seqs_seconds)}


def ego_rpe(frames, gt_tcw):
    """Relative pose error of the ego track against the renderer's ground truth, over
    consecutive frames (the reference's camera RPE, Tracking.cc:1319-1345, taken per frame step):
    the translation (m) and rotation (deg) of (G_b G_a^-1)^-1 (T_b T_a^-1); median, p95 and max."""
    te, re = [], []
    for a in range(len(frames) - 1):
        Ta = np.asarray(frames[a]["Tcw"], np.float64)
        Tb = np.asarray(frames[a + 1]["Tcw"], np.float64)
        Ga, Gb = np.asarray(gt_tcw[a], np.float64), np.asarray(gt_tcw[a + 1], np.float64)
        E = np.linalg.inv(Gb @ np.linalg.inv(Ga)) @ (Tb @ np.linalg.inv(Ta))
        te.append(float(np.linalg.norm(E[:3, 3])))
        re.append(float(np.degrees(np.arccos(np.clip((np.trace(E[:3, :3]) - 1) / 2, -1, 1)))))
    if not te:
        return None
    q = lambda v, p: round(float(np.percentile(v, p)), 6)  # noqa: E731
    return {"frames": len(te) + 1, "trans_m_median": q(te, 50), "trans_m_p95": q(te, 95),
            "trans_m_max": round(max(te), 6), "rot_deg_median": q(re, 50),
            "rot_deg_p95": q(re, 95), "rot_deg_max": round(max(re), 6)}


def rank_parity(args, seqs, seq_frames, rank, wls):
    """The oracle over the first --rank-parity-frames frames of each of this rank's sequences
    (one core each, after the timed region), compared with the GPU's frames: a compact parity
    record per sequence for multi-sequence and multi-rank lines."""
    from concurrent.futures import ThreadPoolExecutor
    from multimot_track_amd import shard
    from oracle import compare, oracle as O
    O.build()
    K = len(wls)
    n = min([args.rank_parity_frames] + [len(f) for f in seq_frames])
    frames = [[seq_frame_numpy(seqs[k], i) for i in range(n)] for k in range(K)]

    def one(k):  # the oracle's C calls release the GIL: one thread per sequence
        wl = wls[k]
        tr = O.Tracker(wl["width"], wl["height"], (721.5377, 721.5377, 609.5593, 172.8540),
                       387.5744, 0, wl["nfeatures"])
        if args.vocabulary:
            tr.set_vocabulary(args.vocabulary)
        ofr = [tr.track(f["bgr"], f["disp"], f["flow"], f["sem"]) for f in frames[k]]
        rec = compare.parity_record(seq_frames[k][:n], ofr)
        return {"rank": rank, "sequence": k, "workload": wl["name"], "seed": wl["seed"],
                "frames": rec["frames"], "first_divergent_frame": rec["first_divergent_frame"],
                "max_pose_diff": rec["max_pose_diff"],
                "int_mismatch_frames": rec["int_mismatch_frames"],
                "lm_stop_flips": rec["lm_stop_flips"],
                "map_tracked": sum(int(d["map_state"] == 1) for d in seq_frames[k][:n])}
    with ThreadPoolExecutor(max_workers=K) as ex:
        return list(ex.map(one, range(K)))


# ------------------------------------------------------------------ dry rehearsal
def run_dry(args, rank, world):
    """The rank logic of the real run on CPU (gloo): per-rank seed, barrier-bracketed timed
    region, MAX-over-ranks time, SUM of frames, world-size-based n_gpus."""
    import torch
    import torch.distributed as dist
    from multimot_track_amd import shard
    dev = torch.device("cpu")
    C, K = args.chunk, args.seqs_per_gpu
    wls = [shard.workload(args.config, rank * K + k) for k in range(K)]
    seeds = [wl["seed"] for wl in wls]
    rsteps = []
    for wl in wls:
        n = None if wl["length"] is None else int(wl["length"] * args.dry_length_scale)
        rsteps.append(shard.rank_steps(n, C, args.warmup, args.steps))
    R = max(1, args.ranks_per_gpu)
    step_s = 0.01 * (rank + 1)  # rank r's stand-in step cost
    for _ in range(max(w for w, _ in rsteps)):
        time.sleep(step_s)
    shard.barrier(world, dev)
    t0 = time.perf_counter()
    for _ in range(max(t for _, t in rsteps)):
        time.sleep(step_s)
    shard.barrier(world, dev)
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, world, dev)
    frames_all = shard.sum_over_ranks(sum(t for _, t in rsteps) * C, world, dev)
    mine = [dict(name=wl["name"], seed=wl["seed"], width=wl["width"], height=wl["height"],
                 timed_steps=t) for wl, (_, t) in zip(wls, rsteps)]
    all_seeds = [None] * world
    all_wl = [None] * world
    if world > 1:
        dist.all_gather_object(all_seeds, seeds)
        dist.all_gather_object(all_wl, mine)
    else:
        all_seeds = [seeds]
        all_wl = [mine]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(frames_all / elapsed, 2),
                          "unit": "frames/s", "n_gpus": world // R, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "u8", "data": "dry run (no GPU work)",
                          "config": {"workload": "dry", "config": args.config,
                                     "chunk_frames": C, "sequences_per_gpu": K * R,
                                     "parallelism": "dp%d" % (world // R), "seeds": all_seeds,
                                     "ranks": all_wl, "frames_all": frames_all}}), flush=True)


# ------------------------------------------------------------------ main
def main(argv=None):
    args = parse_args(argv)
    R = max(1, args.ranks_per_gpu)
    if (args.gpus > 1 or R > 1) and "WORLD_SIZE" not in os.environ:
        return self_launch(args)

    # GPU_MAX_HW_QUEUES (hardware queues the HIP runtime multiplexes a process's streams onto,
    # default 4; every context drives 5 streams) is read at HIP init: set before torch touches the
    # device.  More queues measured slower (profiles/r05_hwq_sweep.txt).
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.hw_queues))
    import torch
    import torch.distributed as dist
    from multimot_track_amd import shard

    rank, world, local = shard.rank_env()
    if world > 1:
        # several ranks on one GPU: RCCL wants one rank per device, so the (tiny) barrier and
        # reductions go through gloo on host tensors
        dist.init_process_group("gloo" if args.dry or R > 1 else "nccl", init_method="env://")
        world = dist.get_world_size()
    if args.dry:
        run_dry(args, rank, world)
        if world > 1:
            dist.destroy_process_group()
        return 0

    import multimot_track_amd as M
    from multimot_track_amd import scene

    local //= R  # the GPU of this rank (R ranks per GPU)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rdev = torch.device("cpu") if R > 1 else dev  # where the cross-rank reductions run
    n_gpus = world // R

    C, K = args.chunk, args.seqs_per_gpu
    # this rank's sequences (shard.workload: C3 by default; C4 / C5 per-rank geometry and length)
    wls = [shard.workload(args.config, rank * K + k) for k in range(K)]
    if args.config == "C3":  # the C3 knobs stay overridable
        for wl in wls:
            wl.update(width=args.width, height=args.height, nfeatures=args.nfeatures,
                      objects=args.objects)
    rsteps = [shard.rank_steps(wl["length"], C, args.warmup, args.steps) for wl in wls]
    W, H, NF = wls[0]["width"], wls[0]["height"], wls[0]["nfeatures"]
    t_gen = time.perf_counter()

    def render(seed, n, objects=None, wl=None):
        # in pieces of 400 frames (each frame is rendered on its own, so the sequence is the
        # same), with a progress line on stderr for long runs under a profiler
        wl = wl or wls[0]
        objects = wl["objects"] if objects is None else objects
        parts = []
        for s0 in range(0, n, 400):
            parts.append(scene.kitti_like_sequence(min(400, n - s0), wl["width"], wl["height"],
                                                   n_objects=objects, seed=seed, device=dev,
                                                   start=s0, lanes=wl["lanes"]))
            print("rank %d: rendered %d / %d frames" % (rank, s0 + len(parts[-1]["Tcw"]), n),
                  file=sys.stderr, flush=True)
        out = {k: torch.cat([p[k] for p in parts]) for k in ("bgr", "disp", "flow", "mask")}
        out["Tcw"] = np.concatenate([p["Tcw"] for p in parts])
        if wl["parts"] > 1 and objects > 0:  # C5: rigid column bands of the boxes (8 motions)
            out["mask"] = scene.split_label_bands(out["mask"], wl["parts"])
        return out

    seqs = [render(wl["seed"], (w + t) * C, wl=wl) for wl, (w, t) in zip(wls, rsteps)]
    seq = seqs[0]
    torch.cuda.synchronize(dev)
    t_gen = time.perf_counter() - t_gen

    cfgs = [M.kitti03_config(wl["width"], wl["height"], wl["nfeatures"], max_batch=C,
                             device_id=local) for wl in wls]
    cfg = cfgs[0]
    ctxs = [M.Context(c) for c in cfgs]
    for c in ctxs:
        if args.vocabulary:
            c.load_vocabulary(args.vocabulary)
    ctx = ctxs[0]
    if not args.immediate:
        for c in ctxs:
            c.set_deferred_objects(True)
    lv = ctx.levels()
    # dedicated (non-default) streams: the library launches on them and records its HIP events
    # on them; torch.cuda.synchronize below waits for all of them
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    torch.cuda.set_stream(streams[0])

    def step_k(k, i, s=None, c=None):
        sl = slice(i * C, (i + 1) * C)
        s = s if s is not None else seqs[k]
        c = c if c is not None else ctxs[k]
        return c.track_chunk_device(s["bgr"][sl], s["disp"][sl], s["flow"][sl], s["mask"][sl],
                                    streams[k].cuda_stream, parse=False)

    pool = None
    if K > 1:  # one host thread per sequence (the C-ABI calls release the GIL)
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=K)

    def step(i, timed):  # the raw results of this rank's sequences that still have chunk i
        ks = [k for k in range(K) if (i < rsteps[k][1] if timed else i < rsteps[k][0])]
        idx = [(rsteps[k][0] + i) if timed else i for k in ks]
        if pool is None:
            return {k: step_k(k, j) for k, j in zip(ks, idx)}
        futs = {k: pool.submit(step_k, k, j) for k, j in zip(ks, idx)}
        return {k: f.result() for k, f in futs.items()}

    warm = [step(i, False) for i in range(max(w for w, _ in rsteps))]
    torch.cuda.synchronize(dev)
    ctx.profile_enable(True)
    ctx.profile_read(reset=True)
    shard.barrier(world, dev)
    t0 = time.perf_counter()
    results = [step(i, True) for i in range(max(t for _, t in rsteps))]
    flushed = [[] for _ in range(K)]
    if not args.immediate:  # the timed frames' last object motions, inside the timed region
        if pool is None:
            flushed = [ctx.flush_objects()]
        else:
            flushed = [f.result() for f in [pool.submit(c.flush_objects) for c in ctxs]]
    torch.cuda.synchronize(dev)
    shard.barrier(world, dev)
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    elapsed = shard.max_over_ranks(elapsed, world, rdev)
    frames_all = shard.sum_over_ranks(sum(t for _, t in rsteps) * C, world, rdev)

    # per-frame outputs of every sequence (sanity: every timed frame tracked by the map, objects
    # found); a line whose timed frames are not all tracked is marked invalid
    seq_frames = [assemble([r[k] for r in warm + results if k in r], C, flushed[k])
                  for k in range(K)]
    all_frames = seq_frames[0]
    timed_frames = all_frames[rsteps[0][0] * C:]
    n_obj_last = len(timed_frames[-1]["objects"]) if timed_frames else 0
    tracked_rank = sum(int(d["initialized"]) for k, f in enumerate(seq_frames)
                       for d in f[rsteps[k][0] * C:])
    tracked = int(shard.sum_over_ranks(tracked_rank, world, rdev))
    lost_first = [next((rsteps[k][0] * C + i for i, d in enumerate(f[rsteps[k][0] * C:])
                        if not d["initialized"]), None) for k, f in enumerate(seq_frames)]
    gt = seq["Tcw"][len(all_frames) - 1]
    ego_err = float(np.abs(all_frames[-1]["Tcw"] - gt).max())
    rpe = ego_rpe(all_frames[rsteps[0][0] * C:], seq["Tcw"][rsteps[0][0] * C:len(all_frames)])
    rank_wl = [dict(name=wl["name"], seed=wl["seed"], width=wl["width"], height=wl["height"],
                    orb_features=wl["nfeatures"], objects=wl["objects"] * wl["parts"],
                    frames_timed=rsteps[k][1] * C, length=wl["length"])
               for k, wl in enumerate(wls)]
    if world > 1:
        g = [None] * world
        dist.all_gather_object(g, rank_wl)
        rank_wl = [r for x in g for r in x]
    mc = ctx.map_counters()
    local_mapping = {k: int(mc[k]) for k in ("n_ba", "n_fused", "n_culled", "n_ba_erased",
                                             "ba_trials", "ba_edges", "ba_pts", "ba_max_opt",
                                             "fuse_launches", "fuse_queries", "fuse_relaunches",
                                             "d2_split_fallbacks")}
    local_mapping["vocabulary"] = os.path.basename(args.vocabulary) if args.vocabulary else None
    if args.vocabulary:  # the BoW steps inside the timed region (TRK, relocalisation, CNMP)
        local_mapping["bow"] = ctx.bow_counters()
    if mc["lm_us"] > 0:  # host wall times, collected with MMT_MAP_PROFILE=1
        for k in ("lm_us", "ba_us", "fuse_us"):
            local_mapping[k] = round(float(mc[k]), 1)
    local_mapping["keyframes_last_frame"] = int(timed_frames[-1]["n_keyframes"])
    local_mapping["mappoints_last_frame"] = int(timed_frames[-1]["n_mappoints"])
    # the timed contexts are done: the legs below run beside no other context of this process (a
    # context's streams share the process's hardware queues with every other context's)
    for c in ctxs:
        c.close()
    # every rank's sequences checked against the oracle over their first frames (several sequences
    # or ranks: the N = 1 line's CPU leg below checks the one sequence over more frames)
    rank_par = None
    if (world > 1 or K > 1) and args.rank_parity_frames > 0:
        rank_par = rank_parity(args, seqs, seq_frames, rank, wls)
        if world > 1:
            gathered = [None] * world
            dist.all_gather_object(gathered, rank_par)
            rank_par = [r for g in gathered for r in g]

    if rank == 0:
        value = frames_all / elapsed
        launch_ms = prof["orb_ms"] / max(prof["orb_launches"], 1)
        bytes_per_launch = C * b_orb(W, H, NF, lv["level_w"], lv["level_h"])
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        key = "%dx%d_n%d_b%d" % (W, H, NF, C)
        traffic = load_traffic(args.traffic_file, key)
        cpu, parity, c2, single = None, None, None, None
        if world == 1 and args.single_frames > 0 and args.config == "C3":
            # the reference-shaped call pattern: one frame per call (rgbd_tum.cc's loop), objects
            # deferred; a fresh sequence context over the frames after the timed region
            ns = args.single_frames
            s1 = render(shard.sequence_seed(1003, 0), ns + 8)
            sctx = M.Context(M.kitti03_config(W, H, NF, max_batch=8, device_id=local))
            if args.vocabulary:
                sctx.load_vocabulary(args.vocabulary)
            sctx.set_deferred_objects(True)
            for i in range(8):  # initialisation and warm-up
                sctx.track_chunk_device(s1["bgr"][i:i + 1], s1["disp"][i:i + 1],
                                        s1["flow"][i:i + 1], s1["mask"][i:i + 1],
                                        streams[0].cuda_stream, parse=False)
            torch.cuda.synchronize(dev)
            ts = time.perf_counter()
            for i in range(8, 8 + ns):
                sctx.track_chunk_device(s1["bgr"][i:i + 1], s1["disp"][i:i + 1],
                                        s1["flow"][i:i + 1], s1["mask"][i:i + 1],
                                        streams[0].cuda_stream, parse=False)
            sctx.flush_objects()
            torch.cuda.synchronize(dev)
            ts = time.perf_counter() - ts
            single = {"value": round(ns / ts, 2), "unit": "frames/s",
                      "ms_per_frame": round(ts / ns * 1e3, 4), "frames": ns,
                      "sample": "frames 8-%d of the C3 sequence, one frame per "
                                "mmt_track_rgbd_chunk_device call, deferred object results, "
                                "flush inside the timed region" % (7 + ns)}
            sctx.close()
            del s1
        if world == 1 and args.c2_steps > 0 and args.config == "C3":
            # C2 (ego only): same camera and sequence seed, mask == 0
            nc2 = (1 + args.c2_steps) * C
            s2 = render(shard.sequence_seed(1003, 0), nc2, objects=0)
            c2ctx = M.Context(cfg)
            if args.vocabulary:
                c2ctx.load_vocabulary(args.vocabulary)
            step_k(0, 0, s2, c2ctx)
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            for i in range(args.c2_steps):
                step_k(0, 1 + i, s2, c2ctx)
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter() - t2
            c2 = {"value": round(args.c2_steps * C / t2, 2), "unit": "frames/s",
                  "frames": args.c2_steps * C, "timed_from": C}
            c2ctx.close()
        if world == 1 and not args.no_cpu:
            gpu_frames = all_frames
            timed_from = rsteps[0][0] * C
            n_t, t_t, parity = cpu_leg(args, seq, gpu_frames, timed_from, W, H, NF)
            fps1 = n_t / t_t if t_t > 0 else 0.0
            cpu = {"value": round(fps1, 3), "unit": "frames/s", "cores": 1,
                   "kind": "port", "cpu_model": cpu_model(), "nproc": os.cpu_count(),
                   "sample": "frames %d-%d of the same C3 sequence (the GPU timed region starts "
                             "at frame %d), full per-frame tracking (oracle/track_ref.cpp), one "
                             "thread pinned to one core, %.1f s of CPU time, after an untimed "
                             "run-up over frames 0-%d" % (timed_from, timed_from + n_t - 1,
                                                          timed_from, t_t, timed_from - 1)}
            if c2 is not None:
                from oracle import oracle as O
                tr2 = O.Tracker(W, H, (721.5377, 721.5377, 609.5593, 172.8540), 387.5744, 0, NF)
                if args.vocabulary:
                    tr2.set_vocabulary(args.vocabulary)
                n2, tt2 = 0, 0.0
                while tt2 < 5.0 and n2 < nc2:
                    f = seq_frame_numpy(s2, n2)
                    ta = time.perf_counter()
                    tr2.track(f["bgr"], f["disp"], f["flow"], f["sem"])
                    tt2 += time.perf_counter() - ta
                    n2 += 1
                cpu["c2_value"] = round(n2 / tt2, 3)
                cpu["c2_sample"] = "frames 0-%d of the C2 sequence, one core, %.1f s" % (n2 - 1,
                                                                                         tt2)
            if args.cpu_seqs > 0:
                cpu["multi"] = cpu_multi_leg(args, lambda sd, n: render(sd, n), W, H, NF, fps1)
        frames_timed = int(frames_all)
        out = {
            "metric": METRIC,
            "value": round(value, 2), "unit": "frames/s", "n_gpus": n_gpus,
            "frames_timed": frames_timed, "frames_tracked": tracked,
            "valid": tracked == frames_timed,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic (seeded ray-cast street sequence, exact depth/flow/"
                                   "labels, KITTI-03 camera), resident in HBM",
            "config": {"workload": WORKLOADS[args.config] % (wls[0]["objects"] * wls[0]["parts"]),
                       "config": args.config, "ranks": rank_wl, "ego_rpe": rpe,
                       "width": W, "height": H, "orb_features": NF, "chunk_frames": C,
                       "sequences_per_gpu": K * R, "ranks_per_gpu": R,
                       "parallelism": "dp%d" % n_gpus if R == 1 else "dp%d x %d ranks per GPU" % (
                           n_gpus, R),
                       "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "frames_tracked": tracked, "objects_last_frame": n_obj_last,
                       "ego_abs_err_last_frame": round(ego_err, 5),
                       "scene_render_s": round(t_gen, 2), "c2": c2,
                       "object_results": "immediate" if args.immediate else "deferred",
                       "local_mapping": local_mapping, "one_frame_per_call": single},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "kernel": "batched ORB window (k_gray_depth, k_resize, k_fast, "
                                   "k_octree, k_blur, k_orient_desc) over %d frames" % C,
                         "launch_ms": round(launch_ms, 4), "bytes_per_launch": bytes_per_launch,
                         "orb_share_of_step": round(prof["orb_ms"] / (elapsed * 1e3), 4)},
            "cpu_baseline": cpu,
            "parity": parity if parity is None else dict(parity, ego_rpe=rpe),
            "rank_parity": rank_par,
        }
        if tracked != frames_timed:
            out["invalid_reason"] = (
                "map tracking lost on %d of the %d timed frames (first lost frame per sequence of "
                "rank 0: %s): the timed region did not run the tracked path on every frame"
                % (frames_timed - tracked, frames_timed, lost_first))
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    if pool is not None:
        pool.shutdown()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
