"""GPU parity of the HIP ORB extractor against the CPU oracle (bit-exact: keypoint records and
descriptors compared as bytes), stage by stage so a failure names the kernel."""
import numpy as np
import pytest

import multimot_track_amd as M
from multimot_track_amd import synthetic

pytestmark = pytest.mark.gpu


def _ctx(w, h, nf, batch=1):
    return M.Context(M.kitti03_config(w, h, nf, max_batch=batch))


def _levels_from_flat(flat, ctx):
    lv = ctx.levels()
    out, off = [], 0
    for w, h in zip(lv["level_w"], lv["level_h"]):
        out.append(flat[off:off + w * h].reshape(h, w))
        off += w * h
    return out


def _compare(k, d, kr, dr, tag):
    if len(k) != len(kr):
        bad_lv = [l for l in range(8) if (k["octave"] == l).sum() != (kr["octave"] == l).sum()]
        raise AssertionError("%s: %d vs %d keypoints; level counts differ at %s" %
                             (tag, len(k), len(kr), bad_lv))
    kb, krb = k.view(np.uint8).reshape(len(k), 28), kr.view(np.uint8).reshape(len(kr), 28)
    rows = np.where((kb != krb).any(1))[0]
    assert len(rows) == 0, "%s: %d keypoint records differ, first %s vs %s" % (
        tag, len(rows), k[rows[:3]], kr[rows[:3]])
    drow = np.where((d != dr).any(1))[0]
    assert len(drow) == 0, "%s: %d descriptors differ (first idx %s)" % (tag, len(drow), drow[:5])


def _check_stages(ctx, gray, O, tag):
    pyr_ref = O.pyramid(gray)
    pyr = _levels_from_flat(ctx.debug_fetch(0), ctx)
    for l, (a, b) in enumerate(zip(pyr, pyr_ref)):
        nd = int((a != b).sum())
        assert nd == 0, "%s: pyramid level %d differs in %d px" % (tag, l, nd)
    blur = _levels_from_flat(ctx.debug_fetch(1), ctx)
    for l, (a, b) in enumerate(zip(blur, pyr_ref)):
        ref = O.blur7(b)
        nd = int((a != ref).sum())
        assert nd == 0, "%s: blurred level %d differs in %d px" % (tag, l, nd)
    err = ctx.debug_fetch(6).view(np.int32)[0]
    assert err == 0, "device error flags %d" % err


def test_orb_kitti_bit_exact(kitti_frames, oracle_mod):
    for nf in (2000, 4000):
        ctx = _ctx(1242, 375, nf)
        for i, fr in enumerate(kitti_frames):
            gray = oracle_mod.gray_from_bgr(fr["bgr"])
            k, d = ctx.orb_extract(gray)
            _check_stages(ctx, gray, oracle_mod, "kitti f%d n%d" % (i, nf))
            kr, dr = oracle_mod.orb_extract(gray, nf)
            _compare(k, d, kr, dr, "kitti f%d n%d" % (i, nf))
        ctx.close()


@pytest.mark.parametrize("w,h,nf,seed", [(1242, 375, 2000, 1), (1241, 376, 4000, 2),
                                         (1226, 370, 4000, 3), (640, 480, 1000, 4),
                                         (1920, 1080, 8000, 5), (400, 260, 300, 6)])
def test_orb_synthetic_sizes_bit_exact(w, h, nf, seed, oracle_mod):
    ctx = _ctx(w, h, nf)
    gray = synthetic.gray_frame(h, w, seed)
    k, d = ctx.orb_extract(gray)
    _check_stages(ctx, gray, oracle_mod, "synth %dx%d" % (w, h))
    kr, dr = oracle_mod.orb_extract(gray, nf)
    _compare(k, d, kr, dr, "synth %dx%d n%d" % (w, h, nf))


def test_too_small_image_is_rejected():
    # the reference divides by zero when a level has no FAST cell row (ORBextractor.cc:784-787)
    with pytest.raises(M.MmtError):
        _ctx(333, 211, 300)


def test_orb_edge_cases(oracle_mod):
    w, h = 640, 480
    ctx = _ctx(w, h, 1000)
    rng = np.random.default_rng(9)
    cases = {
        "constant": np.full((h, w), 77, np.uint8),
        "noise": rng.integers(0, 256, (h, w), dtype=np.uint8),        # very many corners
        "low_contrast": (120 + rng.integers(0, 12, (h, w))).astype(np.uint8),  # minTh fallback
        "checker": ((np.indices((h, w)).sum(0) // 5) % 2 * 200 + 20).astype(np.uint8),
        "half_black": np.where(np.arange(w)[None, :] < w // 2, 0,
                               synthetic.gray_frame(h, w, 3)).astype(np.uint8),
    }
    for name, g in cases.items():
        k, d = ctx.orb_extract(g)
        kr, dr = oracle_mod.orb_extract(g, 1000)
        _compare(k, d, kr, dr, name)
    assert len(ctx.orb_extract(cases["constant"])[0]) == 0


def test_orb_batch_matches_single(kitti_frames, oracle_mod):
    ctx = _ctx(1242, 375, 2000, batch=4)
    grays = [oracle_mod.gray_from_bgr(f["bgr"]) for f in kitti_frames]
    grays = grays + [synthetic.gray_frame(375, 1242, 11), grays[0]]
    outs = ctx.orb_extract_batch(grays)
    for i, (g, (k, d)) in enumerate(zip(grays, outs)):
        kr, dr = oracle_mod.orb_extract(g, 2000)
        _compare(k, d, kr, dr, "batch frame %d" % i)


def test_orbextractor_mirror_api(kitti_frames, oracle_mod):
    ex = M.ORBextractor(2000, 1.2, 8, 20, 7)
    gray = oracle_mod.gray_from_bgr(kitti_frames[1]["bgr"])
    k, d = ex(gray, None)
    kr, dr = oracle_mod.orb_extract(gray, 2000)
    _compare(k, d, kr, dr, "mirror")
    assert ex.GetLevels() == 8
    assert np.allclose(ex.GetScaleFactors(), oracle_mod.orb_config(2000)["scale"])


def test_device_error_flags_are_reported(kitti_frames, oracle_mod):
    """A tripped octree guard (pass limit, node capacity, output truncation) surfaces as
    MMT_EDEVICE from the next synchronous call and from mmt_orb_device_status, then clears."""
    ctx = _ctx(1242, 375, 2000)
    gray = oracle_mod.gray_from_bgr(kitti_frames[0]["bgr"])
    ctx.orb_extract(gray)
    ctx.orb_device_status()  # clean
    ctx.debug_orb_raise(4)
    with pytest.raises(M.MmtError, match="octree-output-truncated"):
        ctx.orb_extract(gray)
    k, d = ctx.orb_extract(gray)  # cleared by the report
    kr, dr = oracle_mod.orb_extract(gray, 2000)
    _compare(k, d, kr, dr, "after flag reset")
    ctx.debug_orb_raise(1 | 2)
    with pytest.raises(M.MmtError, match="octree-pass-guard octree-node-capacity"):
        ctx.orb_device_status()
    ctx.orb_device_status()
    ctx.close()
