"""One frame per mmt_track_rgbd_chunk_device call on the bench's C3 sequence (bench.py's
one_frame_per_call leg: frames 8.. of seed 1003, deferred object results), timed per call and
split into the calls that created a keyframe (LocalMapping runs inside them) and the others.
Usage: python tools/one_frame_bench.py [--frames 256] [--start 8]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--start", type=int, default=8)
    ap.add_argument("--objects", type=int, default=3)
    ap.add_argument("--immediate", action="store_true", help="object results at every call")
    a = ap.parse_args()
    import torch
    import multimot_track_amd as M
    from multimot_track_amd import scene, shard
    dev = torch.device("cuda:0")
    n = a.start + a.frames
    s = scene.kitti_like_sequence(n, 1242, 375, n_objects=a.objects,
                                  seed=shard.sequence_seed(1003, 0), device=dev)
    ctx = M.Context(M.kitti03_config(1242, 375, 2000, max_batch=8))
    ctx.set_deferred_objects(not a.immediate)
    st = torch.cuda.Stream(dev).cuda_stream  # a stream of the caller's, as bench.py's leg

    def call(i):
        return ctx.track_chunk_device(s["bgr"][i:i + 1], s["disp"][i:i + 1], s["flow"][i:i + 1],
                                      s["mask"][i:i + 1], st, parse=False)

    for i in range(a.start):
        call(i)
    torch.cuda.synchronize(dev)
    t, kf = [], []
    t_all = time.perf_counter()
    for i in range(a.start, n):
        t0 = time.perf_counter()
        raw = call(i)
        t.append(time.perf_counter() - t0)
        kf.append(int(raw[0][0].new_keyframe))
    if not a.immediate:
        ctx.flush_objects()
    torch.cuda.synchronize(dev)
    t_all = time.perf_counter() - t_all
    t, kf = np.array(t) * 1e3, np.array(kf, bool)
    print("one frame per call: %d frames (%d-%d) in %.1f ms = %.3f ms/frame (%.1f frames/s)" %
          (a.frames, a.start, n - 1, t_all * 1e3, t_all * 1e3 / a.frames, a.frames / t_all))
    print("  keyframe calls: %d, mean %.3f ms, median %.3f ms; sum %.1f ms = %.3f ms per frame" %
          (kf.sum(), t[kf].mean() if kf.any() else 0, np.median(t[kf]) if kf.any() else 0,
           t[kf].sum(), t[kf].sum() / a.frames))
    print("  other calls: %d, mean %.3f ms, median %.3f ms, p90 %.3f ms" %
          ((~kf).sum(), t[~kf].mean(), np.median(t[~kf]), np.percentile(t[~kf], 90)))
    ctx.close()


if __name__ == "__main__":
    main()
