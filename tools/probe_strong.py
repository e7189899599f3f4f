"""Strong-scaling proxy on one GPU: time for rank r's share (chunks r, r+N, ...) of the C3 frame
vs the full frame, per N (the work one GPU of an N-GPU C4 split does), on the bench's path
(rt_render_ex: RGBA8 rows stored into a page-locked whole-frame buffer) and device-only."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
sc = (scenes.scene_c3 if cfg == "c3" else scenes.scene_c5)(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
stream = torch.cuda.current_stream()
out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
fb = M.pinned_array((H, W, 4), np.uint8)


def t_dev(first, step, k=30):
    for _ in range(3):
        eng.render_device(0, 0, first, step, stream=stream.cuda_stream, out_rgba_ptr=out.data_ptr())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        eng.render_device(0, 0, first, step, stream=stream.cuda_stream, out_rgba_ptr=out.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k


def t_host(first, step, k=30):
    for _ in range(3):
        eng.render_into(0, first, step, rgba=fb, frame_layout=True)
    t = time.perf_counter()
    kms = 0.0
    for _ in range(k):
        kms += eng.render_into(0, first, step, rgba=fb, frame_layout=True).kernel_ms
    return (time.perf_counter() - t) * 1e3 / k, kms / k


fd = t_dev(0, 1)
fh, fk = t_host(0, 1)
print(f"full frame: device {fd:.4f} ms, render_into {fh:.4f} ms (kernel {fk:.4f})", flush=True)
for n in (2, 4, 8):
    wd = max(t_dev(r, n) for r in range(n))
    hs = [t_host(r, n) for r in range(n)]
    wh = max(h for h, _ in hs)
    wk = max(k for _, k in hs)
    print(f"N={n}: slowest share device {wd:.4f} ms (eff {fd / (n * wd):.3f}); render_into {wh:.4f} ms "
          f"(kernel {wk:.4f}; eff {fh / (n * wh):.3f})", flush=True)
