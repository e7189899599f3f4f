"""Strong-scaling proxy on one GPU: the per-GPU frame time of an N-GPU C4 split is the time of
the slowest rank's share (chunks r, r+N, ...).  Each share is rendered K times through the
bench's path (rt_render_submit / rt_render_wait into page-locked whole-frame buffers, Q renders
in flight) and through rt_render_ex one frame at a time; efficiency = T(full) / (N * T(share))."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
sc = (scenes.scene_c3 if cfg == "c3" else scenes.scene_c5)(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
for kv in filter(None, os.environ.get("PROBE_OPT", "").split(",")):   # e.g. PROBE_OPT=tile_order=100
    k, v = kv.split("=")
    eng.set_option(k, int(v))
W, H = sc.cameras[0].image_resolution
QS = [int(x) for x in os.environ.get("PROBE_Q", "1,4,8").split(",")]
NS = [int(x) for x in os.environ.get("PROBE_N", "2,4,8").split(",")]
Q = max(QS + [4])
fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]
K = int(os.environ.get("PROBE_K", "40"))


def t_pipe(first, step, q):
    submit, wait = eng.frame_pipeline(0, first, step, fbs[:q], frame_layout=True)

    def run():
        pend = collections.deque()
        for k in range(K):
            if len(pend) == q:
                wait(pend.popleft())
            pend.append(submit(k))
        while pend:
            wait(pend.popleft())
    run()
    t = time.perf_counter()
    run()
    return (time.perf_counter() - t) * 1e3 / K


full = {q: t_pipe(0, 1, q) for q in sorted(set(QS + [4]))}
print("full frame ms: " + ", ".join(f"{q} in flight {v:.4f}" for q, v in full.items()), flush=True)
for n in NS:
    for q in QS:
        worst = max(t_pipe(r, n, q) for r in range(n))
        print(f"N={n} {q} in flight: slowest share {worst:.4f} ms/frame -> {full[q] / worst:.2f}x of the same "
              f"pipeline on 1 GPU (eff {full[q] / (n * worst):.3f}); vs 1 GPU at 4 in flight "
              f"{full[4] / worst:.2f}x", flush=True)
