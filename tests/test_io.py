"""CPU tests of the rgbd_mmt drop-in's input decoding (SURVEY §8b drop-in CLI, §8f-2 formats):
libmmt_io.so decodes the reference's own kitti_sample files (PNG image and u16 disparity,
semantic text mask; committed under tests/golden/kitti_raw) to exactly the arrays of the
committed npz fixture, which was decoded independently with PIL/numpy
(tools/make_kitti_fixture.py); .flo, settings and sequence text files round-trip."""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, load_kitti_frame

RAW = os.path.join(GOLDEN, "kitti_raw")
IO_LIB = os.path.join(ROOT, "multimot_track_amd", "libmmt_io.so")


@pytest.fixture(scope="module")
def io():
    if not os.path.exists(IO_LIB):
        from multimot_track_amd import build as B
        B.build()
    L = ctypes.CDLL(IO_LIB)
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    L.mmt_io_read_png.argtypes = [ctypes.c_char_p, ip, ip, ip, ip, ctypes.POINTER(vp)]
    L.mmt_io_read_flo.argtypes = [ctypes.c_char_p, ip, ip, ctypes.POINTER(vp)]
    L.mmt_io_read_mask.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, vp]
    L.mmt_io_read_times.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp), ip]
    L.mmt_io_read_poses.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp), ip]
    L.mmt_io_yaml_float.argtypes = [ctypes.c_char_p, ctypes.c_char_p,
                                    ctypes.POINTER(ctypes.c_double)]
    L.mmt_io_write_png_bgr.argtypes = [ctypes.c_char_p, vp, ctypes.c_int, ctypes.c_int]
    L.mmt_io_free.argtypes = [vp]
    return L


def read_png(io, path):
    w, h, c, d = (ctypes.c_int() for _ in range(4))
    p = ctypes.c_void_p()
    rc = io.mmt_io_read_png(path.encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c),
                            ctypes.byref(d), ctypes.byref(p))
    if rc != 0:
        return rc, None
    dt = np.uint8 if d.value == 1 else np.uint16
    n = w.value * h.value * c.value
    a = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8 if d.value == 1
                                                              else ctypes.c_uint16)), (n,))
    out = a.astype(dt).reshape(h.value, w.value, c.value).copy()
    io.mmt_io_free(p)
    return 0, out


def test_png_decodes_kitti_image_and_disparity(io):
    fr = load_kitti_frame(0)
    rc, bgr = read_png(io, os.path.join(RAW, "image_000000.png"))
    assert rc == 0 and np.array_equal(bgr, fr["bgr"])  # imread: BGR order
    rc, disp = read_png(io, os.path.join(RAW, "depth_000000.png"))
    assert rc == 0 and disp.shape[2] == 1 and disp.dtype == np.uint16
    assert np.array_equal(disp[:, :, 0], fr["disp"])


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "I;16", "LA"])
def test_png_modes_match_pil(io, tmp_path, mode):
    from PIL import Image
    rng = np.random.default_rng(3)
    h, w = 37, 53
    if mode == "I;16":
        arr = rng.integers(0, 65535, (h, w), dtype=np.uint16)
        img = Image.fromarray(arr)  # uint16 -> mode I;16
        want = arr[:, :, None]
    else:
        ch = {"RGB": 3, "RGBA": 4, "L": 1, "LA": 2}[mode]
        # smooth + noisy content so the encoder picks several filter types
        base = (np.add.outer(np.arange(h), np.arange(w))[:, :, None] * 3 +
                rng.integers(0, 40, (h, w, ch))).astype(np.uint8)
        img = Image.fromarray(base[:, :, 0] if ch == 1 else base, mode)
        want = base.copy()
        if ch >= 3:
            want[:, :, [0, 2]] = want[:, :, [2, 0]]
    p = str(tmp_path / "x.png")
    img.save(p, optimize=False)
    rc, got = read_png(io, p)
    assert rc == 0 and np.array_equal(got, want)


def test_png_rejects_garbage(io, tmp_path):
    p = tmp_path / "bad.png"
    p.write_bytes(b"not a png at all")
    assert read_png(io, str(p))[0] < 0
    assert read_png(io, str(tmp_path / "missing.png"))[0] < 0


def test_png_writer_round_trips_through_pil_and_the_reader(io, tmp_path):
    """cv::imwrite of a BGR image (rgbd_mmt --viz's feat.png / speed.png / traj.png): PIL reads
    the RGB it stored, and mmt_io_read_png reads back the BGR bytes."""
    from PIL import Image
    rng = np.random.default_rng(5)
    bgr = rng.integers(0, 256, (41, 67, 3), dtype=np.uint8)
    p = str(tmp_path / "w.png")
    assert io.mmt_io_write_png_bgr(p.encode(), bgr.ctypes.data, 67, 41) == 0
    assert np.array_equal(np.asarray(Image.open(p).convert("RGB")), bgr[:, :, ::-1])
    rc, got = read_png(io, p)
    assert rc == 0 and np.array_equal(got, bgr)
    assert io.mmt_io_write_png_bgr(str(tmp_path / "no" / "dir.png").encode(), bgr.ctypes.data,
                                   67, 41) < 0


def test_flo_round_trip(io, tmp_path):
    fr = load_kitti_frame(0)
    flow = fr["flow"]
    h, w = flow.shape[:2]
    p = tmp_path / "f.flo"
    with open(p, "wb") as f:
        f.write(np.float32(202021.25).tobytes() + np.int32(w).tobytes() + np.int32(h).tobytes())
        f.write(flow.astype(np.float32).tobytes())
    ww, hh = ctypes.c_int(), ctypes.c_int()
    ptr = ctypes.c_void_p()
    assert io.mmt_io_read_flo(str(p).encode(), ctypes.byref(ww), ctypes.byref(hh),
                              ctypes.byref(ptr)) == 0
    got = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_float)),
                                (hh.value * ww.value * 2,)).reshape(h, w, 2).copy()
    io.mmt_io_free(ptr)
    assert np.array_equal(got, flow)
    bad = tmp_path / "bad.flo"
    bad.write_bytes(np.float32(1.0).tobytes() + b"\0" * 8)
    assert io.mmt_io_read_flo(str(bad).encode(), ctypes.byref(ww), ctypes.byref(hh),
                              ctypes.byref(ptr)) < 0


def test_mask_loader_filters_labels(io):
    fr = load_kitti_frame(0)  # conftest applies LoadMask's filter to the raw fixture labels
    h, w = fr["sem"].shape
    out = np.full((h, w), -7, np.int32)
    n = io.mmt_io_read_mask(os.path.join(RAW, "semantic_000000.txt").encode(), h, w,
                            out.ctypes.data_as(ctypes.c_void_p))
    assert n == h and np.array_equal(out, fr["sem"])


def test_sequence_text_files(io, tmp_path):
    (tmp_path / "times.txt").write_text("0000\n5.000000e-02\n\n1.000000e-01\n")
    (tmp_path / "pose.txt").write_text("0 " + " ".join(str(float(v)) for v in np.eye(4).ravel())
                                       + "\n1 " + " ".join(str(v + 0.5) for v in range(16)) + "\n")
    (tmp_path / "s.yaml").write_text("%YAML:1.0\n# c\nCamera.fx: 721.5377\nCamera.bf: 387.5744 "
                                     "# comment\nORBextractor.nFeatures: 4000\n")
    p, n = ctypes.c_void_p(), ctypes.c_int()
    assert io.mmt_io_read_times(str(tmp_path / "times.txt").encode(), ctypes.byref(p),
                                ctypes.byref(n)) == 0
    t = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_double)), (n.value,)).copy()
    io.mmt_io_free(p)
    assert np.array_equal(t, [0.0, 0.05, 0.1])
    assert io.mmt_io_read_poses(str(tmp_path / "pose.txt").encode(), ctypes.byref(p),
                                ctypes.byref(n)) == 0
    P = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)),
                              (n.value * 16,)).reshape(-1, 16).copy()
    io.mmt_io_free(p)
    assert n.value == 2 and np.array_equal(P[0], np.eye(4).ravel())
    assert np.allclose(P[1], np.arange(16) + 0.5)
    v = ctypes.c_double()
    y = str(tmp_path / "s.yaml").encode()
    assert io.mmt_io_yaml_float(y, b"Camera.bf", ctypes.byref(v)) == 0 and v.value == 387.5744
    assert io.mmt_io_yaml_float(y, b"ORBextractor.nFeatures", ctypes.byref(v)) == 0
    assert v.value == 4000
    assert io.mmt_io_yaml_float(y, b"Camera.fy", ctypes.byref(v)) != 0


def test_cli_usage_and_missing_sequence(tmp_path):
    import subprocess
    exe = os.path.join(ROOT, "multimot_track_amd", "rgbd_mmt")
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stderr
    (tmp_path / "s.yaml").write_text("Camera.fx: 1\n")
    r = subprocess.run([exe, "voc", str(tmp_path / "s.yaml"), str(tmp_path)], capture_output=True,
                       text=True)
    assert r.returncode == 1 and "No images" in r.stderr
