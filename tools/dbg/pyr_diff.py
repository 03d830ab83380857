"""Where does the GPU pyramid differ from the oracle?  Prints, per level, the count of differing
pixels, their row/column ranges and a few samples (GPU value, oracle value)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import multimot_track_amd as M  # noqa: E402
from conftest import load_kitti_frame  # noqa: E402
from oracle import oracle as O  # noqa: E402

ctx = M.Context(M.kitti03_config(1242, 375, 2000))
gray = O.gray_from_bgr(load_kitti_frame(0)["bgr"])
ctx.orb_extract(gray)
flat = ctx.debug_fetch(0)
bflat = ctx.debug_fetch(1)
lv = ctx.levels()
ref = O.pyramid(gray)
off = 0
for l, (w, h) in enumerate(zip(lv["level_w"], lv["level_h"])):
    a = flat[off:off + w * h].reshape(h, w)
    b = bflat[off:off + w * h].reshape(h, w)
    off += w * h
    for name, got, exp in (("pyr", a, ref[l]), ("blur", b, O.blur7(ref[l]))):
        d = np.argwhere(got != exp)
        if len(d) == 0:
            print("level %d %s ok" % (l, name))
            continue
        ys, xs = d[:, 0], d[:, 1]
        print("level %d %s: %d px differ, rows %d..%d cols %d..%d" %
              (l, name, len(d), ys.min(), ys.max(), xs.min(), xs.max()))
        print("  distinct rows (first 20):", np.unique(ys)[:20].tolist())
        print("  distinct cols (first 40):", np.unique(xs)[:40].tolist())
        for y, x in d[:6]:
            print("  (%d,%d) gpu %d ref %d" % (y, x, got[y, x], exp[y, x]))
ctx.close()
