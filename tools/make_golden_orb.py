"""Generate tests/golden/orb_kitti.npz: oracle ORB outputs on the kitti_sample frames (full
keypoints+descriptors of frame 0 at N=2000, sha256 digests for frames 0-4 at N=2000/4000).
These pin the oracle against accidental drift; they are produced by the CPU restatement because
the reference itself cannot be built here (parity status)."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_kitti_frame, kitti_meta  # noqa: E402
from oracle import oracle as O  # noqa: E402

out = {}
for i in range(kitti_meta()["frames"]):
    g = O.gray_from_bgr(load_kitti_frame(i)["bgr"])
    for nf in (2000, 4000):
        k, d = O.orb_extract(g, nf)
        h = hashlib.sha256()
        h.update(np.ascontiguousarray(k).tobytes())
        h.update(np.ascontiguousarray(d).tobytes())
        out["digest_f%d_n%d" % (i, nf)] = np.array(h.hexdigest())
        if i == 0 and nf == 2000:
            out["kps_f0_n2000"] = k
            out["desc_f0_n2000"] = d
np.savez_compressed(os.path.join(ROOT, "tests", "golden", "orb_kitti.npz"), **out)
print("ok", len(out))
