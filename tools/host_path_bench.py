"""PCIe-inclusive rate of the host-buffer entry point mmt_track_rgbd (System::TrackRGBD's
per-frame form: host BGR / disparity / flow / labels in, one frame per call, ORB batch of one)
on the bench's C3 sequence.  Usage: host_path_bench.py [frames] [warmup]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import multimot_track_amd as M  # noqa: E402
from multimot_track_amd import scene  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda:0")
seq = scene.kitti_like_sequence(n + warm, 1242, 375, n_objects=3, seed=1003, device=dev)
frames = scene.to_numpy_frames(seq)  # host copies, as a caller's decoded frames
ctx = M.Context(M.kitti03_config(1242, 375, 2000))
for f in frames[:warm]:
    ctx.track(f["bgr"], f["disp"], f["flow"], f["sem"])
t0 = time.perf_counter()
for f in frames[warm:]:
    ctx.track(f["bgr"], f["disp"], f["flow"], f["sem"])
dt = time.perf_counter() - t0
print("host-buffer mmt_track_rgbd: %d frames (%d-%d) in %.3f s = %.1f frames/s" %
      (n, warm, warm + n - 1, dt, n / dt), flush=True)
ctx.close()
