"""Do consecutive frames overlap on the GPU?  A C4 share (chunks r::N) or the whole C3 frame,
rendered K times through rt_render_device on 1, 2 or 4 HIP streams in turn (each stream its
own output buffer); wall time per frame."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import myraytracer_amd as M  # noqa: E402
from myraytracer_amd import scenes  # noqa: E402

sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache"))
W, H = sc.cameras[0].image_resolution
K = 40
for ns in (1, 4, 8):
    eng = M.RayTracerEngine(sc)
    streams = [torch.cuda.Stream() for _ in range(ns)]
    outs = [torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(ns)]
    for n, first in ((1, 0), (8, 5)):
        def run():
            for k in range(K):
                q = k % ns
                eng.render_device(0, 0, first, n, stream=streams[q].cuda_stream, out_rgba_ptr=outs[q].data_ptr(),
                                  slot=0)
            torch.cuda.synchronize()
        run()
        t = time.perf_counter()
        run()
        ms = (time.perf_counter() - t) * 1e3 / K
        print(f"streams {ns}: share {first}::{n}: {ms:.4f} ms per frame", flush=True)
    eng.close()
