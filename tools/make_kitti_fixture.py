"""Convert the reference's only data fixture (kitti_sample/, 5 KITTI-03 frames) into compressed
npz + json under tests/golden/kitti_sample/, so tests on the GPU box (which has no
/root/reference) read exactly the same input bytes.

Decoding mirrors rgbd_tum.cc: imread(UNCHANGED) gives BGR u8 (:122) and a u16 disparity PNG
(:123, converted to float by :124); readOpticalFlow gives HxWx2 float32 (:129); the semantic
text mask is kept raw (LoadMask's label<4 filter, rgbd_tum.cc:335, is applied by the loader).
Data only -- no reference source is copied.
"""
import json
import os
import sys

import numpy as np
from PIL import Image

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/kitti_sample"
dst = sys.argv[2] if len(sys.argv) > 2 else "tests/golden/kitti_sample"
os.makedirs(dst, exist_ok=True)


def read_flo(path):
    with open(path, "rb") as f:
        magic = np.frombuffer(f.read(4), np.float32)[0]
        assert abs(magic - 202021.25) < 1e-3, magic
        w, h = np.frombuffer(f.read(8), np.int32)
        data = np.frombuffer(f.read(int(w) * int(h) * 8), np.float32)
    return data.reshape(int(h), int(w), 2).copy()


n = 0
while os.path.exists(os.path.join(src, "image", "%06d.png" % n)):
    rgb = np.array(Image.open(os.path.join(src, "image", "%06d.png" % n)).convert("RGB"))
    bgr = rgb[:, :, ::-1].copy()
    disp = np.array(Image.open(os.path.join(src, "depth", "%06d.png" % n)))
    assert disp.dtype in (np.uint16, np.int32), disp.dtype
    disp = disp.astype(np.uint16)
    flow = read_flo(os.path.join(src, "flow", "%06d.flo" % n))
    sem = np.loadtxt(os.path.join(src, "semantic", "%06d.txt" % n), dtype=np.int32)
    assert sem.shape == bgr.shape[:2]
    np.savez_compressed(os.path.join(dst, "frame_%06d.npz" % n), bgr=bgr, disp=disp, flow=flow,
                        sem=sem)
    n += 1

def floats(line):
    return [float(t) for t in line.split()]

meta = {
    "frames": n,
    "times": [float(l) for l in open(os.path.join(src, "times.txt")) if l.strip()],
    "pose_gt": [floats(l) for l in open(os.path.join(src, "pose_gt.txt")) if l.strip()],
    "object_pose": [floats(l) for l in open(os.path.join(src, "object_pose.txt")) if l.strip()],
    "settings": {},
}
for line in open(os.path.join(src, "kitti03.yaml")):
    line = line.split("#")[0].strip()
    if ":" in line and not line.startswith("%"):
        k, v = line.split(":", 1)
        try:
            meta["settings"][k.strip()] = float(v)
        except ValueError:
            pass
json.dump(meta, open(os.path.join(dst, "meta.json"), "w"), indent=1)
print("frames:", n)
