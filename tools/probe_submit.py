"""Host cost of rt_render_submit / rt_render_wait: time spent inside each call (Python-side
wall clock around the ctypes call) for a C4 share with Q renders in flight."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(8)]
for (first, step), Q in (((0, 1), 4), ((5, 8), 2), ((5, 8), 4), ((5, 8), 8)):
    submit, wait = eng.frame_pipeline(0, first, step, fbs[:Q], frame_layout=True)
    for rep in range(2):
        ts, tw, pend = [], [], collections.deque()
        t0 = time.perf_counter()
        for k in range(60):
            if len(pend) == Q:
                a = time.perf_counter(); wait(pend.popleft()); tw.append(time.perf_counter() - a)
            a = time.perf_counter(); pend.append(submit(k)); ts.append(time.perf_counter() - a)
        while pend:
            wait(pend.popleft())
        tot = (time.perf_counter() - t0) * 1e3 / 60
        print(f"share {first}::{step}, {Q} in flight: {tot:.4f} ms/frame; submit {np.mean(ts) * 1e3:.4f} ms "
              f"(p90 {np.percentile(ts, 90) * 1e3:.4f}), wait {np.mean(tw) * 1e3:.4f} ms", flush=True)
