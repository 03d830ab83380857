"""GPU test of the rgbd_mmt drop-in: the reference's sequence layout is written
from the kitti_sample fixture (PNG image + u16 disparity, .flo, semantic text, times.txt,
pose_gt.txt, settings yaml), rgbd_mmt tracks it through libmmt, and its poses equal the
C-ABI's mmt_track_rgbd on the same decoded frames bit for bit and the CPU oracle within 1e-4."""
import json
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

from conftest import KITTI, ROOT, kitti_meta, load_kitti_frame

pytestmark = pytest.mark.gpu


def write_sequence(d):
    meta = kitti_meta()
    for sub in ("image", "depth", "flow", "semantic"):
        os.makedirs(os.path.join(d, sub))
    for i in range(meta["frames"]):
        raw = np.load(os.path.join(KITTI, "frame_%06d.npz" % i))
        Image.fromarray(raw["bgr"][:, :, ::-1].copy(), "RGB").save(
            os.path.join(d, "image", "%06d.png" % i))
        Image.fromarray(raw["disp"]).save(os.path.join(d, "depth", "%06d.png" % i))
        h, w = raw["disp"].shape
        with open(os.path.join(d, "flow", "%06d.flo" % i), "wb") as f:
            f.write(np.float32(202021.25).tobytes() + np.int32(w).tobytes() +
                    np.int32(h).tobytes() + raw["flow"].astype(np.float32).tobytes())
        np.savetxt(os.path.join(d, "semantic", "%06d.txt" % i), raw["sem"], fmt="%d")
    with open(os.path.join(d, "times.txt"), "w") as f:
        f.write("\n".join("%e" % t for t in meta["times"]) + "\n")  # longer than the data
    with open(os.path.join(d, "pose_gt.txt"), "w") as f:
        for row in meta["pose_gt"]:
            f.write("%d " % int(row[0]) + " ".join("%.9f" % v for v in row[1:]) + "\n")
    with open(os.path.join(d, "settings.yaml"), "w") as f:
        f.write("%YAML:1.0\n")
        for k, v in meta["settings"].items():
            f.write("%s: %s\n" % (k, repr(v)))
    return meta["frames"]


def test_cli_tracks_sequence_like_the_c_abi(tmp_path, oracle_mod):
    import multimot_track_amd as M
    n = write_sequence(str(tmp_path))
    out = str(tmp_path / "poses.txt")
    exe = os.path.join(ROOT, "multimot_track_amd", "rgbd_mmt")
    r = subprocess.run([exe, "ORBvoc.txt", str(tmp_path / "settings.yaml"), str(tmp_path),
                        "--nfeatures", "2000", "--poses", out], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Images in the sequence: %d" % n in r.stdout
    assert r.stdout.count("relative pose error of estimated camera pose, t:") == 2 * (n - 1)
    assert "median tracking time:" in r.stdout and "mean tracking time:" in r.stdout
    cli = np.loadtxt(out)[:, 1:].reshape(-1, 4, 4).astype(np.float32)
    assert len(cli) == n
    ctx = M.Context(M.kitti03_config(nfeatures=2000))
    tr = oracle_mod.Tracker(1242, 375, (ctx.cfg.fx, ctx.cfg.fy, ctx.cfg.cx, ctx.cfg.cy),
                            ctx.cfg.bf, 0, 2000)
    for i in range(n):
        f = load_kitti_frame(i)
        g = ctx.track(f["bgr"], f["disp"], f["flow"], f["sem"])
        o = tr.track(f["bgr"], f["disp"], f["flow"], f["sem"])
        assert np.abs(cli[i] - g["Tcw"]).max() <= 1e-6  # printed with 9 decimals
        assert np.abs(cli[i] - o["Tcw"]).max() < 1e-4
    ctx.close()
