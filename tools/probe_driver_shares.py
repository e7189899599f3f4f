"""The driver's multi-GPU measurement, rehearsed one share at a time on one GPU: for N ranks, each
rank's share of the C3 frame (8-row chunks r, r+N, ...) rendered the way bench.py times it - W
warmup frames, then K frames with 16 in flight between a device sync on both sides - and the
slowest share's time is what the N-GPU line would report (max over ranks).  Render options
(tile_order, ...) as NAME=VALUE arguments; PROBE_N (default 1,2,4,8), PROBE_K (20), PROBE_W (5),
PROBE_REPS (3: the median of repeated timings of each share)."""
import collections
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import myraytracer_amd as M
from myraytracer_amd import _abi as A
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
for kv in sys.argv[1:]:
    k, v = kv.split("=")
    eng.set_option(k, int(v))
W, H = sc.cameras[0].image_resolution
Q = A.RT_MAX_IN_FLIGHT
fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]
K = int(os.environ.get("PROBE_K", "20"))
WU = int(os.environ.get("PROBE_W", "5"))
REPS = int(os.environ.get("PROBE_REPS", "3"))
NS = [int(x) for x in os.environ.get("PROBE_N", "1,2,4,8").split(",")]
rays_frame = None


def share(first, step):
    submit, wait = eng.frame_pipeline(0, first, step, fbs, frame_layout=True)

    def run(n):
        pend = collections.deque()
        st = None
        for k in range(n):
            if len(pend) == Q:
                st = wait(pend.popleft())
            pend.append(submit(k))
        while pend:
            st = wait(pend.popleft())
        return st
    run(WU)
    ts = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t = time.perf_counter()
        st = run(K)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3 / K)
    return statistics.median(ts), int(st.primary_rays + st.shadow_rays_traced)


opts = " ".join(sys.argv[1:]) or "defaults"
for n in NS:
    per = [share(r, n) for r in range(n)]
    worst = max(p[0] for p in per)
    rays = sum(p[1] for p in per)
    print(f"[{opts}] N={n}: slowest share {worst:.4f} ms/frame (shares {min(p[0] for p in per):.4f}.."
          f"{worst:.4f}) -> {rays / worst / 1e3:.1f} Mrays/s whole job", flush=True)
eng.close()
