"""The profiled ORB window of the tracker (k_gray_depth + the ORB launch sequence, as bench.py's
roofline) on the reference's kitti_sample frames, cycled into one 32-frame chunk that is tracked
`reps` times: light on host-side work, so rocprofv3 --pmc passes stay short.
Usage: orb_window_bench.py [batch] [reps]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import multimot_track_amd as M  # noqa: E402
from conftest import load_kitti_frame  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
W, H, NF = 1242, 375, 2000
dev = torch.device("cuda:0")
fr = [load_kitti_frame(i) for i in range(5)]


def stack(key, dtype=None):
    a = np.stack([fr[i % 5][key] for i in range(B)])
    return torch.from_numpy(a if dtype is None else a.view(dtype)).to(dev).contiguous()


bgr, disp = stack("bgr"), stack("disp", np.int16)
flow, sem = stack("flow"), stack("sem")
ctx = M.Context(M.kitti03_config(W, H, NF, max_batch=B))
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
ctx.track_chunk_device(bgr, disp, flow, sem, stream.cuda_stream, parse=False)
torch.cuda.synchronize()
ctx.profile_enable(True)
ctx.profile_read(reset=True)
for _ in range(reps):
    ctx.track_chunk_device(bgr, disp, flow, sem, stream.cuda_stream, parse=False)
torch.cuda.synchronize()
p = ctx.profile_read()
ms = p["orb_ms"] / max(p["orb_launches"], 1)
lv = ctx.levels()
P = int(sum(int(a) * int(b) for a, b in zip(lv["level_w"], lv["level_h"])))
bw = 3 * W * H + 4 * P + 60 * NF + 6 * W * H
print("batch=%d window_ms=%.4f us_per_frame=%.2f GB/s=%.1f frac=%.4f" %
      (B, ms, ms * 1e3 / B, B * bw / (ms * 1e-3) / 1e9, B * bw / (ms * 1e-3) / 8e12), flush=True)
ctx.close()
