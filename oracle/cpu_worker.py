"""One CPU-baseline worker of bench.py (TEST INFRASTRUCTURE: the oracle timed as the reference's
CPU path).  Tracks one sequence, stored by the parent as .npy arrays in `dir`, with the scalar
oracle on one pinned core for about `seconds` of CPU time, and prints one JSON line
{"frames", "seconds", "core"}.  It never touches the GPU (no torch import): the parent renders
the frames on the GPU and starts the workers as child processes.

usage: python -m oracle.cpu_worker DIR CORE SECONDS W H NFEAT [VOCABULARY]"""
import json
import os
import sys
import time

import numpy as np


def main():
    d, core, seconds = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    W, H, nfeat = int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
    if core >= 0 and hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, {core})
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle as O
    bgr = np.load(os.path.join(d, "bgr.npy"), mmap_mode="r")
    disp = np.load(os.path.join(d, "disp.npy"), mmap_mode="r")
    flow = np.load(os.path.join(d, "flow.npy"), mmap_mode="r")
    mask = np.load(os.path.join(d, "mask.npy"), mmap_mode="r")
    K = (721.5377, 721.5377, 609.5593, 172.8540)
    tr = O.Tracker(W, H, K, 387.5744, 0, nfeat)
    if len(sys.argv) > 7 and sys.argv[7]:
        tr.set_vocabulary(sys.argv[7])
    n, t = 0, 0.0
    while t < seconds and n < len(bgr):
        f = (np.ascontiguousarray(bgr[n]), np.ascontiguousarray(disp[n]),
             np.ascontiguousarray(flow[n]), np.ascontiguousarray(mask[n]))
        t0 = time.perf_counter()
        tr.track(*f)
        t += time.perf_counter() - t0
        n += 1
    print(json.dumps({"frames": n, "seconds": t, "core": core}), flush=True)


if __name__ == "__main__":
    main()
