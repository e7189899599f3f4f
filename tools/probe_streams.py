"""Frames in flight: K C3 frames on one stream vs alternating 2 streams (tails overlap)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = 1920, 1080
outs = [torch.empty((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(2)]
streams = [torch.cuda.Stream() for _ in range(2)]
import time


def run(nstreams, k=40):
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(k):
            s = streams[f % nstreams]
            eng.render_device(outs[f % 2].data_ptr(), f % nstreams, 0, 0, 1, stream=s.cuda_stream) \
                if False else eng.render_device(outs[f % 2].data_ptr(), 0, 0, 1, slot=0, stream=s.cuda_stream)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / k
    return ms


for n in (1, 2):
    print(f"streams={n}: {run(n):.4f} ms/frame", flush=True)
