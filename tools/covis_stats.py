"""Covisibility diagnostics of the oracle map on the bench's C3 sequence (CPU, no GPU needed).

Tracks `frames` frames with the oracle (vocabulary on or off), then prints the map's observation
count histogram, the frame span of each point's observing keyframes, and the most observed points
(position, observation count, octaves, the keys' depths): the far points that CreateNewMapPoints
triangulates from keys at disparity 0 (depth inf) show up here.

  python tools/covis_stats.py 250 1      # 250 frames, vocabulary on
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.set_num_threads(4)
    from oracle import oracle as O
    from multimot_track_amd import scene
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 250
    usevoc = (sys.argv[2] if len(sys.argv) > 2 else "1") == "1"
    seq = scene.kitti_like_sequence(n, 1242, 375, n_objects=3, seed=1003, device="cpu")
    fr = scene.to_numpy_frames(seq)
    tr = O.Tracker(1242, 375, (721.5377, 721.5377, 609.5593, 172.8540), 387.5744, 0, 2000)
    if usevoc:
        tr.set_vocabulary(os.path.join(ROOT, "tests", "golden", "test_voc_k10l6.txt"))
    t0 = time.time()
    for i in range(n):
        f = fr[i]
        r = tr.track(f["bgr"], f["disp"], f["flow"], f["sem"])
    print("frames %d in %.1f s: %d keyframes, %d map points" % (n, time.time() - t0,
                                                               r["n_keyframes"], r["n_mappoints"]))
    md = tr.map_dump()
    pi, pf = md["pt_i"], md["pt_f"]
    g = np.where(pi[:, 0] == 0)[0]
    nobs = np.diff(md["obs_start"])
    print("good points %d, non-finite %d" % (len(g), (~np.isfinite(pf[g]).all(1)).sum()))
    print("observations per point (0..19, 20+):", np.bincount(np.minimum(nobs[g], 20)).tolist())
    frameid = md["kf_i"][:, 1]
    span = []
    for j in g:
        s, e = md["obs_start"][j], md["obs_start"][j + 1]
        if e > s:
            ks = md["obs_i"][s:e, 0]
            span.append(frameid[ks].max() - frameid[ks].min())
    span = np.array(span)
    print("frame span of a point's observing keyframes: median %g, p95 %g, max %d" % (
        np.median(span), np.percentile(span, 95), span.max()))
    for j in g[np.argsort(-nobs[g])[:5]]:
        s, e = md["obs_start"][j], md["obs_start"][j + 1]
        print("point %d at %s: %d observations, keyframe frames %d..%d, octaves %s, depths %s" % (
            j, np.round(pf[j, :3], 2).tolist(), nobs[j], frameid[md["obs_i"][s:e, 0]].min(),
            frameid[md["obs_i"][s:e, 0]].max(), md["obs_i"][s:e, 2][:10].tolist(),
            np.round(md["obs_f"][s:e, 2][:6], 2).tolist()))


if __name__ == "__main__":
    main()
