"""Frames in flight: K C3 frames on one stream vs alternating over 2 streams, so that
the drain of frame k (its last, slowest tiles) overlaps the start of frame k+1."""
import os
import sys
import time

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
outs = [torch.empty((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(2)]
streams = [torch.cuda.Stream() for _ in range(2)]


def run(nstreams, k=40):
    best = 1e9
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(k):
            s = streams[f % nstreams]
            eng.render_device(outs[f % 2].data_ptr(), 0, 0, 1, stream=s.cuda_stream)
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3 / k)
    return best


ref = None
for n in (1, 2, 1, 2):
    print(f"{cfg} streams={n}: {run(n):.4f} ms/frame", flush=True)
# the two streams' frames are identical images
a = outs[0].clone()
eng.render_device(outs[1].data_ptr(), 0, 0, 1, stream=streams[1].cuda_stream)
torch.cuda.synchronize()
print("frames identical:", bool(torch.equal(a, outs[1])), flush=True)
