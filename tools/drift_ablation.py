"""Ego-drift ablation on the CPU oracle (VERDICT r5 "next" #2).

Tracks the bench's C3 sequence (seed 1003) with the oracle tracker under one LocalMapping
ablation per process and logs the per-frame pose error against the renderer's ground truth:
  full      the reference's path as pinned
  no_ba     ORACLE_LM_STEPS=5: SearchInNeighbors + KeyFrameCulling, no local BA
  no_fuse   ORACLE_LM_STEPS=6: local BA + KeyFrameCulling, no SearchInNeighbors / Fuse
  no_lm     ORACLE_LM_STEPS=0: ProcessNewKeyFrame + MapPointCulling only
  no_cull   ORACLE_ABLATE=1: no MapPointCulling
  tlr_post  ORACLE_ABLATE=2: Tlr taken after the keyframe's LocalMapping (round 4's order)
  depth_nearest        ORACLE_ABLATE=4: the keys' depth (mvDepth, mvuRight) read at the nearest
                       pixel instead of the truncated one (Frame.cc:1041-1062's at<float>(v, u))
  no_ba_depth_nearest  both
  level_centre         ORACLE_ABLATE=8: level-l keypoints at their pixel centre's level-0 position
                       ((x + 0.5) s - 0.5) instead of x s (ORBextractor.cc:1100-1104)
  aa3, aa3_no_ba       the same sequence with box-filtered colour (3 x 3 sub-pixel rays per pixel,
                       scene.SequenceRenderer aa): does texture aliasing (the fbm's finest octaves
                       are above the pixel Nyquist rate beyond about 20 m) feed the BA keypoints
                       that do not stay on one surface point?
  static, static_no_ba the same sequence without its three moving boxes (the ego motion, the
                       street and the seed unchanged): do the map points that the moving boxes'
                       keys create drive the drift through the local BA?
Frames are rendered on the GPU (scene.py) and copied to the host; the oracle runs on the host
cores, one process per configuration.  Output: one JSON per configuration with, every 100 frames,
the camera-centre error of the final pose (after the flow solve) and of the map-branch pose, the
per-frame relative pose error (translation of T_rel vs the ground truth's, and its rotation angle)
as median / p95 over the frames so far, and at the end the keyframe poses' centre errors (after
every local BA).

  python tools/drift_ablation.py --frames 3200 --configs full,no_ba --out gpurun_out/drift
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "full": {},
    "no_ba": {"ORACLE_LM_STEPS": "5"},
    "no_fuse": {"ORACLE_LM_STEPS": "6"},
    "no_lm": {"ORACLE_LM_STEPS": "0"},
    "no_cull": {"ORACLE_ABLATE": "1"},
    "tlr_post": {"ORACLE_ABLATE": "2"},
    "depth_nearest": {"ORACLE_ABLATE": "4"},
    "no_ba_depth_nearest": {"ORACLE_ABLATE": "4", "ORACLE_LM_STEPS": "5"},
    "level_centre": {"ORACLE_ABLATE": "8"},
    "aa3": {},
    "aa3_no_ba": {"ORACLE_LM_STEPS": "5"},
    "static": {},
    "static_no_ba": {"ORACLE_LM_STEPS": "5"},
}
N_OBJECTS = {"static": 0, "static_no_ba": 0}
AA = {"aa3": 3, "aa3_no_ba": 3}


def centre(T):
    T = np.asarray(T, np.float64)
    return -T[:3, :3].T @ T[:3, 3]


def rel_errors(Ta, Tb, Ga, Gb):
    """Relative pose error of the step a -> b: translation (m) and rotation (deg) of
    (Gb Ga^-1)^-1 (Tb Ta^-1)."""
    E = np.linalg.inv(Gb @ np.linalg.inv(Ga)) @ (Tb @ np.linalg.inv(Ta))
    ang = np.degrees(np.arccos(np.clip((np.trace(E[:3, :3]) - 1) / 2, -1, 1)))
    return float(np.linalg.norm(E[:3, 3])), float(ang)


def worker(args):
    import torch
    from multimot_track_amd import scene
    from oracle import oracle as O
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    W, H = 1242, 375
    tr = O.Tracker(W, H, (721.5377, 721.5377, 609.5593, 172.8540), 387.5744, 0, 2000)
    rows, rte, rre, rte_map = [], [], [], []
    prev = None
    t0 = time.time()
    out = {"config": args.config, "env": CONFIGS[args.config], "frames": args.frames,
           "seed": args.seed}
    lost = []
    for s0 in range(0, args.frames, 200):
        n = min(200, args.frames - s0)
        seq = scene.kitti_like_sequence(n, W, H, n_objects=N_OBJECTS.get(args.config, 3),
                                        seed=args.seed, device=dev, start=s0,
                                        aa=AA.get(args.config, 1))
        fr = scene.to_numpy_frames(seq)
        for i in range(n):
            f = fr[i]
            g = np.asarray(seq["Tcw"][i], np.float64)
            r = tr.track(f["bgr"], f["disp"], f["flow"], f["sem"])
            T = r["Tcw"].astype(np.float64)
            Tm = r["Tcw_map"].astype(np.float64)
            k = s0 + i
            if r["map_state"] != 1:
                lost.append(k)
            if prev is not None and r["initialized"]:
                a, b = rel_errors(prev[0], T, prev[2], g)
                rte.append(a)
                rre.append(b)
                rte_map.append(rel_errors(prev[1], Tm, prev[2], g)[0])
            prev = (T, Tm, g)
            if k % 100 == 99 or k == args.frames - 1:
                rows.append({"frame": k, "centre_err": float(np.linalg.norm(centre(T) - centre(g))),
                             "centre_err_map": float(np.linalg.norm(centre(Tm) - centre(g))),
                             "abs_err_max_entry": float(np.abs(T - g).max()),
                             "rte_median": float(np.median(rte)), "rte_p95": float(np.percentile(rte, 95)),
                             "rre_median_deg": float(np.median(rre)),
                             "rre_p95_deg": float(np.percentile(rre, 95)),
                             "rte_map_median": float(np.median(rte_map)),
                             "n_keyframes": r["n_keyframes"], "lost_frames": len(lost),
                             "wall_s": round(time.time() - t0, 1)})
                print(args.config, json.dumps(rows[-1]), flush=True)
        del seq, fr
    sc = scene.StreetScene(n_objects=N_OBJECTS.get(args.config, 3), seed=args.seed)  # the keyframes' ground truth
    m = tr.map_dump()
    kf_err = []
    for k in range(len(m["kf_i"])):
        if m["kf_i"][k][2]:  # bad
            continue
        fid = int(m["kf_i"][k][1])
        Twc = np.asarray(sc.Twc(fid), np.float64)
        kf_err.append((fid, float(np.linalg.norm(centre(m["kf_T"][k].reshape(4, 4)) - Twc[:3, 3]))))
    out["rows"] = rows
    out["lost_frames"] = lost[:50]
    out["n_lost"] = len(lost)
    out["map_stats"] = tr.map_stats()
    out["keyframe_centre_err"] = kf_err[::max(1, len(kf_err) // 40)] + kf_err[-1:]
    with open(args.out + "_%s.json" % args.config, "w") as fh:
        json.dump(out, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3200)
    ap.add_argument("--seed", type=int, default=1003)
    ap.add_argument("--configs", default="full,no_ba,no_fuse,no_lm,no_cull,tlr_post")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "drift"))
    ap.add_argument("--config", default=None, help="(worker) one configuration")
    args = ap.parse_args()
    if args.config:
        return worker(args)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    procs = []
    for c in args.configs.split(","):
        env = dict(os.environ)
        env.update(CONFIGS[c])
        env["OMP_NUM_THREADS"] = "1"
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--config", c,
                                       "--frames", str(args.frames), "--seed", str(args.seed),
                                       "--out", args.out], env=env, cwd=ROOT))
    rc = 0
    for p in procs:
        rc |= p.wait()
    return rc


if __name__ == "__main__":
    sys.exit(main())
