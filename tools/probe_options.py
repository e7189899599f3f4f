"""Kernel time of the C3 (or C5 ...) frame under render-option combinations (rt_scene_set_option,
INTEGRATION.md table), A/B in one process; each combination starts from the defaults.
usage: probe_options.py c3 "xcd_group=4" "wide=0 compact_records=0" ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1]
sc = {"c3": scenes.scene_c3, "c5": scenes.scene_c5, "c3i": scenes.scene_c3_instanced,
      "c3g": scenes.scene_c3_glass, "c2": scenes.scene_c2}[cfg](path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
stream = torch.cuda.current_stream()
out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
DEFAULTS = {}


def t_frame(k=20):
    for _ in range(3):
        eng.render_device(out.data_ptr(), 0, 0, 1, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        eng.render_device(out.data_ptr(), 0, 0, 1, stream=stream.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k


for rep in range(2):
    for combo in sys.argv[2:]:
        for k, v in DEFAULTS.items():
            eng.set_option(k, v)
        for kv in combo.split():
            k, v = kv.split("=")
            DEFAULTS.setdefault(k, eng.get_option(k))
            eng.set_option(k, int(v))
        ms = t_frame()
        import hashlib
        sha = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
        print(f"{cfg} [{combo}] {ms:.4f} ms  frame sha1 {sha}  secondary {eng.collect_stats().secondary_rays}",
              flush=True)
