"""GPU test of the rgbd_mmt drop-in: the reference's sequence layout is written
from the kitti_sample fixture (PNG image + u16 disparity, .flo, semantic text, times.txt,
pose_gt.txt, object_pose.txt, settings yaml), rgbd_mmt tracks it through libmmt, and its poses
equal the C-ABI's mmt_track_rgbd on the same decoded frames bit for bit and the CPU oracle within
1e-4; its per-object speed and relative-pose-error lines equal a float64 restatement over the
C-ABI's object motions and centroids to the printed precision."""
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
    with open(os.path.join(d, "object_pose.txt"), "w") as f:
        for row in meta["object_pose"]:
            f.write("%d %d " % (int(row[0]), int(row[1])) +
                    " ".join("%.9g" % v for v in row[2:]) + "\n")
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
    expected = []
    meta = kitti_meta()
    gt = {int(r[0]): np.array(r[1:], np.float64).reshape(4, 4) for r in meta["pose_gt"]}
    for i in range(n):
        f = load_kitti_frame(i)
        g = ctx.track(f["bgr"], f["disp"], f["flow"], f["sem"])
        o = tr.track(f["bgr"], f["disp"], f["flow"], f["sem"])
        assert np.abs(cli[i] - g["Tcw"]).max() <= 1e-6  # printed with 9 decimals
        assert np.abs(cli[i] - o["Tcw"]).max() < 1e-4
        if i > 0:
            for ob in g["objects"]:
                e = object_eval(ob, gt[i - 1], gt[i], meta["object_pose"], i)
                if e is not None:
                    expected.append(e)
    ctx.close()
    # the per-object evaluation lines (Tracking.cc:2178-2243) against a float64 restatement
    # over the C-ABI's vObjMod and ObjCentre3D_pre (printed with 4 decimals)
    speeds = [l for l in r.stdout.splitlines() if l.startswith("estimated and ground truth")]
    rpes = [l for l in r.stdout.splitlines() if l.startswith("the relative pose error of the "
                                                             "object, t:") and "%" in l]
    assert len(expected) > 0 and len(speeds) == len(expected) == len(rpes)
    for line, rpe, e in zip(speeds, rpes, expected):
        got = [float(v) for v in line.split(":")[1].replace("km/h", " ").split()]
        assert np.allclose(got, e[:3], rtol=1e-3, atol=2e-3), (line, e)
        t_pct = float(rpe.split("t:")[1].split("%")[0])
        assert abs(t_pct - e[3]) <= 1e-3 * max(1.0, abs(e[3])) + 2e-3, (rpe, e)


def _obj_pose(row):
    """Tracking::ObjPoseParsing: R = Ry(ry + pi/2), t = row[6:9]."""
    y = row[9] + 3.1415926 / 2
    P = np.eye(4)
    P[:3, :3] = [[np.cos(y), 0, np.sin(y)], [0, 1, 0], [-np.sin(y), 0, np.cos(y)]]
    P[:3, 3] = row[6:9]
    return P


def object_eval(ob, Tlw_gt, Tcw_gt, rows, i):
    """Speeds (est, gt, |diff|) in km/h and t_rpe/t_gt in % for one object of frame i."""
    rp = [r for r in rows if int(r[0]) == i - 1 and int(r[1]) == ob["sem_label"]]
    rc = [r for r in rows if int(r[0]) == i and int(r[1]) == ob["sem_label"]]
    if not rp or not rc:
        return None
    Lwp = np.linalg.inv(Tlw_gt) @ _obj_pose(np.array(rp[0], np.float64))
    Lwc = np.linalg.inv(Tcw_gt) @ _obj_pose(np.array(rc[0], np.float64))
    H = Lwc @ np.linalg.inv(Lwp)
    sp_gt = np.linalg.norm(Lwp[:3, 3] - Lwc[:3, 3])
    M = ob["motion"].astype(np.float64)
    sp_est = np.linalg.norm(M[:3, 3] - (np.eye(3) - M[:3, :3]) @ ob["centre_pre"])
    E = np.linalg.inv(M) @ H
    t_rpe, t_gt = np.linalg.norm(E[:3, 3]), np.linalg.norm(H[:3, 3])
    return (sp_est * 36, sp_gt * 36, abs(sp_est - sp_gt) * 36, t_rpe / t_gt * 100)


def test_cli_writes_the_visual_artifacts(tmp_path):
    """rgbd_mmt --viz (Tracking.cc:684-878): traj.png (600 x 800, the camera squares in red),
    feat.png and speed.png at the image size for the last frame: feat.png is the image with
    red static samples and label-coloured object samples drawn over it, speed.png the gray
    image with orange ground-truth boxes."""
    n = write_sequence(str(tmp_path))
    exe = os.path.join(ROOT, "multimot_track_amd", "rgbd_mmt")
    vd = tmp_path / "viz"
    vd.mkdir()
    r = subprocess.run([exe, "ORBvoc.txt", str(tmp_path / "settings.yaml"), str(tmp_path),
                        "--nfeatures", "2000", "--viz", str(vd)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    traj = np.asarray(Image.open(vd / "traj.png").convert("RGB"))
    feat = np.asarray(Image.open(vd / "feat.png").convert("RGB"))
    speed = np.asarray(Image.open(vd / "speed.png").convert("RGB"))
    assert traj.shape == (800, 600, 3) and feat.shape == (375, 1242, 3) == speed.shape
    red = (traj[:, :, 0] == 255) & (traj[:, :, 1] == 0) & (traj[:, :, 2] == 0)
    assert red.sum() > 4 * 10 * n // 2  # one square outline per frame
    img = load_kitti_frame(n - 1)["bgr"][:, :, ::-1]
    changed = np.any(feat != img, axis=2)
    assert 200 < changed.sum() < 0.5 * changed.size  # drawn over the image
    orange = (speed[:, :, 0] == 255) & (speed[:, :, 1] == 140) & (speed[:, :, 2] == 0)
    g = speed[:, :, 0] == speed[:, :, 1]
    assert g.mean() > 0.9 and orange.sum() > 0


def test_cli_loads_the_vocabulary_like_system(tmp_path):
    """rgbd_mmt with a loadable DBoW2 vocabulary (System.cc:57-67): "Vocabulary loaded!", and its
    poses equal the C-ABI's with the same vocabulary loaded (TrackReferenceKeyFrame on the second
    frame); a missing file is a warning, not an exit."""
    import multimot_track_amd as M
    from conftest import GOLDEN
    voc = os.path.join(GOLDEN, "test_voc_k10l6.txt")
    n = write_sequence(str(tmp_path))
    out = str(tmp_path / "poses.txt")
    exe = os.path.join(ROOT, "multimot_track_amd", "rgbd_mmt")
    r = subprocess.run([exe, voc, str(tmp_path / "settings.yaml"), str(tmp_path),
                        "--nfeatures", "2000", "--poses", out], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Vocabulary loaded!" in r.stdout and "not loaded" not in r.stderr
    cli = np.loadtxt(out)[:, 1:].reshape(-1, 4, 4).astype(np.float32)
    ctx = M.Context(M.kitti03_config(nfeatures=2000))
    try:
        ctx.load_vocabulary(voc)
        for i in range(n):
            f = load_kitti_frame(i)
            g = ctx.track(f["bgr"], f["disp"], f["flow"], f["sem"])
            assert np.abs(cli[i] - g["Tcw"]).max() <= 1e-6
        assert ctx.bow_counters()["trk"] >= 1
    finally:
        ctx.close()
    r = subprocess.run([exe, str(tmp_path / "missing_voc.txt"), str(tmp_path / "settings.yaml"),
                        str(tmp_path), "--nfeatures", "2000"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "not loaded" in r.stderr
