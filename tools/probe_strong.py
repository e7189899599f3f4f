"""Strong-scaling proxy on one GPU: time for rank r's share (chunks r, r+N, ...) of the C3 frame
vs the full frame, per N (the work one GPU of an N-GPU C4 split does)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = 1920, 1080
stream = torch.cuda.current_stream()
out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")


def t_sel(first, step, k=30):
    for _ in range(3):
        eng.render_device(out.data_ptr(), 0, first, step, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        eng.render_device(out.data_ptr(), 0, first, step, stream=stream.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k


full = t_sel(0, 1)
print(f"full frame: {full:.4f} ms", flush=True)
for n in (2, 4, 8):
    worst = max(t_sel(r, n) for r in range(n))
    print(f"N={n}: slowest rank share {worst:.4f} ms  -> strong-scaling efficiency {full / (n * worst):.3f}", flush=True)
