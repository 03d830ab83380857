"""Batched ORB extraction (mmt_orb_extract_device) on synthetic KITTI-sized frames, for per-kernel
timing under rocprofv3 --kernel-trace --stats.  Usage: orb_microbench.py [batch] [reps]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import multimot_track_amd as M  # noqa: E402
from multimot_track_amd import scene  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
W, H, NF = 1242, 375, 2000
dev = torch.device("cuda:0")
if os.environ.get("ORB_MB_SCENE") == "synthetic":
    seq = scene.kitti_like_sequence(B, W, H, n_objects=3, seed=1003, device=dev)
    bgr = seq["bgr"].cpu().numpy()
else:  # the reference's kitti_sample frames, cycled (few host-side ops: cheap under --pmc)
    KITTI = os.path.join(ROOT, "tests", "golden", "kitti_sample")
    fr = [np.load(os.path.join(KITTI, "frame_%06d.npz" % i))["bgr"] for i in range(5)]
    bgr = np.stack([fr[i % 5] for i in range(B)])
g = (bgr.astype(np.int32) * np.array([4899, 9617, 1868], np.int32)).sum(-1)
gray = torch.from_numpy(((g + 8192) >> 14).astype(np.uint8)).to(dev).contiguous()
ctx = M.Context(M.kitti03_config(W, H, NF, max_batch=B))
cap = ctx.capacity()
kps = torch.empty((B, cap * 28), dtype=torch.uint8, device=dev)
desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
n = torch.empty(B, dtype=torch.int32, device=dev)
stream = torch.cuda.Stream(dev)
torch.cuda.synchronize()


def run():
    rc = M.lib().mmt_orb_extract_device(ctx.handle, gray.data_ptr(), B, W * H, kps.data_ptr(),
                                        desc.data_ptr(), cap, n.data_ptr(), stream.cuda_stream)
    assert rc == 0, M.lib().mmt_last_error(ctx.handle)


run()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record(stream)
for _ in range(reps):
    run()
ev1.record(stream)
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1) / reps
lv = ctx.levels()
P = int(sum(int(a) * int(b) for a, b in zip(lv["level_w"], lv["level_h"])))
borb = 3 * W * H + 4 * P + 60 * NF
print("batch=%d ms_per_launch=%.3f us_per_frame=%.2f GB/s=%.1f frac=%.4f kps_mean=%.1f" %
      (B, ms, ms * 1e3 / B, B * borb / (ms * 1e-3) / 1e9, B * borb / (ms * 1e-3) / 8e12,
       n.float().mean().item()), flush=True)
