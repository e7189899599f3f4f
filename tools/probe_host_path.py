"""rt_render host-buffer variants on C3 (batch count, copy engine vs host-mapped stores)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa: F401

import myraytracer_amd as M
from myraytracer_amd import scenes

sc = scenes.scene_c3(path_dir=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scenes_cache"))
eng = M.RayTracerEngine(sc)
pin, _ = eng.alloc_frame(0, 0, 1, rgba=False)
pag = np.zeros_like(pin)
ref, _, st = eng.render_rows(0, 0, 1, False)
rays = st.primary_rays + st.shadow_rays


def run(out, k=8):
    eng.render_rows(0, 0, 1, False, out=out)
    t0 = time.perf_counter()
    for _ in range(k):
        eng.render_rows(0, 0, 1, False, out=out)
    ms = (time.perf_counter() - t0) * 1e3 / k
    assert np.array_equal(out, ref)
    return ms


for zc in (0, 1):                                   # render options zerocopy / batches
    for nb in (1, 2, 4, 8):
        eng.set_option("zerocopy", zc)
        eng.set_option("batches", nb)
        ms = run(pin)
        print(f"pinned zerocopy={zc} batches={nb}: {ms:.3f} ms  {rays / ms / 1e3:.0f} Mrays/s", flush=True)
eng.set_option("zerocopy", 0)
for nb in (2, 4, 8):
    eng.set_option("batches", nb)
    ms = run(pag)
    print(f"pageable batches={nb}: {ms:.3f} ms  {rays / ms / 1e3:.0f} Mrays/s", flush=True)
