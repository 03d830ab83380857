"""Interleaved A/B of environment settings on one rendered sequence: the bench's C3 (and C2)
workload tracked ROUNDS times per setting, settings alternating, each run in a fresh context
(every knob the library reads at context creation or per call takes effect), frames/s per run and
the median per setting.  Removes the box-to-box noise of separate bench runs.
Usage: python tools/ab_interleave.py [--rounds 3] [--steps 6] [--chunk 128] [--c2] 'default' 'VAR=v,VAR2=w' ..."""
import argparse
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("settings", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=128)
    ap.add_argument("--objects", type=int, default=3)
    a = ap.parse_args()
    import torch
    import multimot_track_amd as M
    from multimot_track_amd import scene
    dev = torch.device("cuda", 0)
    W, H, NF, C = 1242, 375, 2000, a.chunk
    n = (a.warmup + a.steps) * C
    parts = []
    for s0 in range(0, n, 400):
        parts.append(scene.kitti_like_sequence(min(400, n - s0), W, H, n_objects=a.objects,
                                               seed=1003, device=dev, start=s0))
        print("rendered %d / %d" % (s0 + len(parts[-1]["Tcw"]), n), file=sys.stderr, flush=True)
    seq = {k: torch.cat([p[k] for p in parts]) for k in ("bgr", "disp", "flow", "mask")}
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    base_env = dict(os.environ)
    res = {s: [] for s in a.settings}
    for r in range(a.rounds):
        for s in a.settings:
            os.environ.clear()
            os.environ.update(base_env)
            if s != "default":
                for kv in s.split(","):
                    k, v = kv.split("=", 1)
                    os.environ[k] = v
            ctx = M.Context(M.kitti03_config(W, H, NF, max_batch=C, device_id=0))

            def step(i):
                sl = slice(i * C, (i + 1) * C)
                return ctx.track_chunk_device(seq["bgr"][sl], seq["disp"][sl], seq["flow"][sl],
                                              seq["mask"][sl], stream.cuda_stream, parse=False)
            for i in range(a.warmup):
                step(i)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(a.steps):
                step(a.warmup + i)
            torch.cuda.synchronize(dev)
            fps = a.steps * C / (time.perf_counter() - t0)
            ctx.close()
            res[s].append(fps)
            print("round %d %-40s %8.1f fps" % (r, s, fps), flush=True)
    os.environ.clear()
    os.environ.update(base_env)
    for s in a.settings:
        print("%-40s median %8.1f  runs %s" % (s, statistics.median(res[s]),
                                               " ".join("%.1f" % v for v in res[s])))


if __name__ == "__main__":
    main()
