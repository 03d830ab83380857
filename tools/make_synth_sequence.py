"""Write a synthetic sequence in the reference's on-disk layout (rgbd_tum.cc LoadData :213-312):
image/%06d.png (RGB), depth/%06d.png (u16 disparity x 256), flow/%06d.flo (Middlebury),
semantic/%06d.txt (one text line of labels per row), times.txt, pose_gt.txt and settings.yaml
(kitti03.yaml's camera), from the bench's ray-cast street scene (multimot_track_amd/scene.py).
object_pose.txt is left empty (the evaluation lines need KITTI object annotations).  For timing
the rgbd_mmt drop-in end to end.

Usage: python tools/make_synth_sequence.py OUT_DIR NFRAMES [--objects 3] [--seed 1003] [--device cuda]
"""
import argparse
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multimot_track_amd import scene  # noqa: E402

SETTINGS = {"Camera.fx": 721.5377, "Camera.fy": 721.5377, "Camera.cx": 609.5593,
            "Camera.cy": 172.854, "Camera.k1": 0.0, "Camera.k2": 0.0, "Camera.p1": 0.0,
            "Camera.p2": 0.0, "Camera.width": 1242, "Camera.height": 375, "Camera.fps": 10.0,
            "Camera.bf": 387.5744, "Camera.RGB": 1, "ThDepth": 40.0,
            "ORBextractor.nFeatures": 2000, "ORBextractor.scaleFactor": 1.2,
            "ORBextractor.nLevels": 8, "ORBextractor.iniThFAST": 20,
            "ORBextractor.minThFAST": 7}


def mask_text(sem):
    """LoadMask's format: `cols` integers per line, separated by spaces (labels < 10 here)."""
    sem = np.asarray(sem)
    assert sem.min() >= 0 and sem.max() < 10
    h, w = sem.shape
    buf = np.full((h, 2 * w), ord(" "), np.uint8)
    buf[:, 0::2] = sem.astype(np.uint8) + ord("0")
    buf[:, -1] = ord("\n")
    return buf.tobytes()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("nframes", type=int)
    ap.add_argument("--objects", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1003)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--piece", type=int, default=100, help="frames rendered per batch")
    a = ap.parse_args()
    for sub in ("image", "depth", "flow", "semantic"):
        os.makedirs(os.path.join(a.out, sub), exist_ok=True)
    W, H = SETTINGS["Camera.width"], SETTINGS["Camera.height"]
    poses = []
    for s0 in range(0, a.nframes, a.piece):
        n = min(a.piece, a.nframes - s0)
        seq = scene.kitti_like_sequence(n, W, H, n_objects=a.objects, seed=a.seed,
                                        device=a.device, start=s0)
        for j, f in enumerate(scene.to_numpy_frames(seq)):
            i = s0 + j
            Image.fromarray(f["bgr"][:, :, ::-1].copy(), "RGB").save(
                os.path.join(a.out, "image", "%06d.png" % i), compress_level=1)
            Image.fromarray(f["disp"]).save(os.path.join(a.out, "depth", "%06d.png" % i),
                                            compress_level=1)
            with open(os.path.join(a.out, "flow", "%06d.flo" % i), "wb") as fo:
                fo.write(np.float32(202021.25).tobytes() + np.int32(W).tobytes() +
                         np.int32(H).tobytes() + f["flow"].astype(np.float32).tobytes())
            with open(os.path.join(a.out, "semantic", "%06d.txt" % i), "wb") as fo:
                fo.write(mask_text(f["sem"]))
        poses += [np.asarray(T, np.float64) for T in seq["Tcw"]]
        print("rendered %d / %d" % (s0 + n, a.nframes), file=sys.stderr, flush=True)
    with open(os.path.join(a.out, "times.txt"), "w") as f:
        f.write("".join("%e\n" % (0.1 * i) for i in range(a.nframes)))
    with open(os.path.join(a.out, "pose_gt.txt"), "w") as f:
        for i, T in enumerate(poses):
            f.write("%d " % i + " ".join("%.9f" % v for v in T.reshape(16)) + "\n")
    open(os.path.join(a.out, "object_pose.txt"), "w").close()
    with open(os.path.join(a.out, "settings.yaml"), "w") as f:
        f.write("%YAML:1.0\n")
        for k, v in SETTINGS.items():
            f.write("%s: %s\n" % (k, repr(v)))


if __name__ == "__main__":
    main()
