"""Work and divergence counters of one frame (rt_render_device_counted, the COUNT instantiation of
the frame's kernel): wide nodes fetched, triangle tests, wave / lane iterations of the walks by
kind (inner step, leaf run) and the SIMD efficiency they imply.
usage: python3 tools/probe_work.py [c3|c5] [-o file]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "c3"
out_path = sys.argv[sys.argv.index("-o") + 1] if "-o" in sys.argv else None
sc = {"c3": scenes.scene_c3, "c5": scenes.scene_c5}[cfg](path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
img = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
wc = eng.work_counters(img.data_ptr())
torch.cuda.synchronize()
lines = [f"{cfg}: {W}x{H}, one frame, counting launch"]
for name, _ in wc._fields_:
    v = getattr(wc, name)
    lines.append(f"  {name:28s} {list(v) if not isinstance(v, int) else v}")
for k, kind in enumerate(("closest", "any-hit")):
    wi, wl = wc.iter_wave_inner[k], wc.iter_wave_leaf[k]
    li, ll = wc.iter_lane_inner[k], wc.iter_lane_leaf[k]
    ws = wc.iter_wave_scalar[k]
    lines.append(f"  {kind}: inner steps {wi} waves x {li / max(wi, 1):.1f} lanes, leaf runs {wl} waves x "
                 f"{ll / max(wl, 1):.1f} lanes, scalar inner steps {ws}")
lines.append(f"  SIMD efficiency closest {wc.lane_steps_closest / max(64 * wc.wave_steps_closest, 1):.3f}, "
             f"any-hit {wc.lane_steps_shadow / max(64 * wc.wave_steps_shadow, 1):.3f}")
text = "\n".join(lines) + "\n"
sys.stdout.write(text)
if out_path:
    open(out_path, "w").write(text)
