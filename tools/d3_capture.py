"""Capture the D3 problem (PoseOptimizationFlow2 of one object) the oracle tracker builds at a
given frame of a synthetic sequence, then solve it with the oracle and the GPU (mmt_pose_flow_solve)
and print both: the tool behind a long-run divergence report.
Usage: python tools/d3_capture.py W H NFEAT SEED OBJECTS FRAME OBJ [--parts P] [--lanes x,d;x,d]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    for k in ("w", "h", "nfeat", "seed", "objects", "frame", "obj"):
        ap.add_argument(k, type=int)
    ap.add_argument("--parts", type=int, default=1)
    ap.add_argument("--lanes", default="")
    a = ap.parse_args()
    import torch
    import multimot_track_amd as M
    from multimot_track_amd import scene
    from oracle import oracle as O
    from synth_problems import K_KITTI
    from test_gpu_track import split_labels
    lanes = [tuple(float(v) for v in p.split(",")) for p in a.lanes.split(";")] if a.lanes else None
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    seq = scene.kitti_like_sequence(a.frame + 1, a.w, a.h, n_objects=a.objects, seed=a.seed,
                                    device=dev, lanes=lanes)
    frames = scene.to_numpy_frames(seq)
    tr = O.Tracker(a.w, a.h, K_KITTI, 387.5744, 0, a.nfeat)
    tr.capture_d3(a.frame, a.obj)
    for f in frames:
        sem = split_labels(f["sem"], a.parts) if a.parts > 1 else f["sem"]
        r = tr.track(f["bgr"], f["disp"], f["flow"], sem)
    P = tr.captured_d3()
    if P is None:
        print("no D3 problem captured")
        return
    ob = r["objects"][a.obj]
    print("oracle tracker: object", a.obj, {k: ob[k] for k in ("label", "n_solve", "n_inliers",
                                                                "iterations")})
    args = (P["obs"], P["flow"], P["depth"], P["tcw_last"], P["init"], 0.01, 0.5, 200, K_KITTI)
    rc, pose_o, st_o = O.flow_solve(*args)
    print("oracle flow_solve: rc", rc, st_o)
    np.savez(os.path.join(ROOT, "gpurun_out", "d3_f%d_o%d.npz" % (a.frame, a.obj)), **P)
    if torch.cuda.is_available():
        ctx = M.Context(M.kitti03_config(a.w, a.h, a.nfeat))
        for env in ({}, {"MMT_LM_SPLIT": "0"},
                    {"MMT_LM_MAX_CAND": "1"}):
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            s, pose_g, st_g = ctx.flow_solve(*args)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
            print("gpu", env or "default", "status", s, st_g, "max pose diff %.3g" %
                  float(np.abs(pose_g - pose_o).max()))
        ctx.close()


if __name__ == "__main__":
    main()
