"""Per-share frame time of an N-GPU C4 split rendered on one GPU (every rank's share, not only
the slowest), with the host time spent inside rt_render_submit / rt_render_wait, to separate
share imbalance from per-frame overhead.  Env: PROBE_N (default 8), PROBE_Q (16), PROBE_K (200),
PROBE_CFG (c3 / c5)."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.environ.get("PROBE_CFG", "c3")
sc = (scenes.scene_c3 if CFG == "c3" else scenes.scene_c5)(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
for kv in filter(None, os.environ.get("PROBE_OPT", "").split(",")):   # e.g. PROBE_OPT=submit_counters=0
    k, v = kv.split("=")
    eng.set_option(k, int(v))
W, H = sc.cameras[0].image_resolution
N = int(os.environ.get("PROBE_N", "8"))
Q = int(os.environ.get("PROBE_Q", "16"))
K = int(os.environ.get("PROBE_K", "200"))
fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]


def run(first, step):
    submit, wait = eng.frame_pipeline(0, first, step, fbs, frame_layout=True)
    for rep in range(2):
        ts = tw = 0.0
        pend = collections.deque()
        t0 = time.perf_counter()
        for k in range(K):
            if len(pend) == Q:
                a = time.perf_counter(); wait(pend.popleft()); tw += time.perf_counter() - a
            a = time.perf_counter(); pend.append(submit(k)); ts += time.perf_counter() - a
        while pend:
            wait(pend.popleft())
        tot = (time.perf_counter() - t0) * 1e3 / K
    return tot, ts * 1e3 / K, tw * 1e3 / K


full = run(0, 1)
print(f"full frame {Q} in flight: {full[0]:.4f} ms/frame (submit {full[1]:.4f}, wait {full[2]:.4f})", flush=True)
res = [run(r, N) for r in range(N)]
for r, (t, s, w) in enumerate(res):
    print(f"N={N} share {r}: {t:.4f} ms/frame (submit {s:.4f}, wait {w:.4f})", flush=True)
tt = [x[0] for x in res]
print(f"N={N}: mean share {np.mean(tt):.4f}, max {max(tt):.4f}; full/N {full[0] / N:.4f}; "
      f"eff(max) {full[0] / (N * max(tt)):.3f}", flush=True)
