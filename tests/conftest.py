import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
KITTI = os.path.join(GOLDEN, "kitti_sample")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libmmt.so")


def load_kitti_frame(i):
    """Frame i of the reference's kitti_sample fixture (rgbd_tum.cc:122-131 decoding):
    BGR u8, disparity*256 u16, flow HxWx2 f32, semantic labels with LoadMask's filter
    (labels 1..3 kept, everything else 0; rgbd_tum.cc:335)."""
    d = np.load(os.path.join(KITTI, "frame_%06d.npz" % i))
    sem = d["sem"]
    sem = np.where((sem != 0) & (sem < 4), sem, 0).astype(np.int32)
    return dict(bgr=d["bgr"], disp=d["disp"], flow=d["flow"], sem=sem)


def kitti_meta():
    return json.load(open(os.path.join(KITTI, "meta.json")))


@pytest.fixture(scope="session")
def kitti_frames():
    return [load_kitti_frame(i) for i in range(kitti_meta()["frames"])]


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build()
    return O
