"""Debug probe: C5 frames through the compacted bounce render (option queue = 1) against the bounce
megakernel (queue = 0) of the same library, in the order the parity test renders them (sampled
chunks, then the full frame), reporting the pixels that differ."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import myraytracer_amd as M
from myraytracer_amd import scenes

sc = scenes.scene_c5(path_dir="scenes_cache")
out = {}
for q in (1, 0):
    eng = M.RayTracerEngine(sc)
    eng.set_option("queue", q)
    for first, step in ((100, 64), (0, 1), (100, 64), (0, 1)):
        rgb, rgba, st = eng.render_rows(0, first, step, True)
        out.setdefault((q, first), []).append((rgb.copy(), st.secondary_rays))
    eng.close()
for first in (100, 0):
    a, sa = out[(0, first)][0]
    for rep in range(2):
        b, sb = out[(1, first)][rep]
        d = np.abs(a - b).max(axis=2)
        ys, xs = np.nonzero(d > 1e-9)
        print("first", first, "rep", rep, "secondary", sa, sb, "bad pixels", len(ys), "max", d.max())
        if len(ys):
            print(" rows", np.unique(ys)[:20], "n rows", len(np.unique(ys)), "cols", np.unique(xs)[:20])
            print(" rows mod 8", np.unique(ys % 8), "cols mod 8", np.unique(xs % 8))
            for y, x in list(zip(ys, xs))[:5]:
                print("  ", y, x, a[y, x], b[y, x])
