"""Where does the public path's extra time go?  C3 frames through rt_render_device with the
RGBA8 image stored (a) into HBM, (b) into page-locked host memory (the kernel's stores cross
PCIe), each (1) back to back on one stream and (2) one launch at a time with a host sync in
between (as rt_render runs), plus rt_render_ex itself (call wall time / kernel events)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import myraytracer_amd as M  # noqa: E402
from myraytracer_amd import scenes  # noqa: E402

sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
dev8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
host8 = M.pinned_array((H, W, 4), np.uint8)
s = torch.cuda.current_stream().cuda_stream


def run(ptr, k=40, sync_each=False):
    for _ in range(3):
        eng.render_device(0, 0, 0, 1, stream=s, out_rgba_ptr=ptr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        eng.render_device(0, 0, 0, 1, stream=s, out_rgba_ptr=ptr)
        if sync_each:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / k


for rep in range(2):
    for name, ptr in (("hbm", dev8.data_ptr()), ("host", host8.ctypes.data)):
        print(f"{name}: back-to-back {run(ptr):.4f} ms/frame, synced each {run(ptr, sync_each=True):.4f} ms/frame",
              flush=True)
    f = eng.frame_renderer(0, 0, 1, rgb=None, rgba=host8, frame_layout=True)
    for _ in range(3):
        f()
    calls, kms = [], []
    t0 = time.perf_counter()
    for _ in range(40):
        st = f()
        calls.append(st.milliseconds)
        kms.append(st.kernel_ms)
    wall = (time.perf_counter() - t0) * 1e3 / 40
    print(f"rt_render_ex: wall {wall:.4f} ms/frame, in-call {np.mean(calls):.4f}, kernel events {np.mean(kms):.4f}",
          flush=True)
