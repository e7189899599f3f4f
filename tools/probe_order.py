"""Tile-order A/B on C3: full frame and the 1/8 share (strong-scaling proxy) per MYRT_ORDER."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache")) if cfg == "c3" else \
    scenes.scene_c5(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
stream = torch.cuda.current_stream()
out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")


def t_sel(first, step, k=20):
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


for order in sys.argv[2:] if len(sys.argv) > 2 else ["0", "1", "2"]:
    os.environ["MYRT_ORDER"] = order
    full = t_sel(0, 1)
    eighth = max(t_sel(r, 8) for r in range(8))
    print(f"{cfg} order={order}: full {full:.4f} ms, slowest 1/8 share {eighth:.4f} ms", flush=True)
