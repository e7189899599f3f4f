"""Per-wave timeline of the C3 megakernel (rt_debug_wave_times): duration distribution, the
number of resident waves over time (the tail), and the most expensive tiles."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import myraytracer_amd as M
from myraytracer_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
FIRST = int(sys.argv[2]) if len(sys.argv) > 2 else 0     # chunk selection (a rank's C4 share)
STEP = int(sys.argv[3]) if len(sys.argv) > 3 else 1
TAG = sys.argv[4] if len(sys.argv) > 4 else "0"       # label of the run
sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache")) if cfg == "c3" else \
    scenes.scene_c5(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
lib = M.load_library()
nw = C.c_int64()
lib.rt_debug_wave_times(eng.handle, 0, 0, FIRST, STEP, C.c_void_p(out.data_ptr()), None, 0, C.byref(nw))
buf = np.zeros(nw.value * 3, np.uint64)
for _ in range(3):   # warm
    lib.rt_debug_wave_times(eng.handle, 0, 0, FIRST, STEP, C.c_void_p(out.data_ptr()),
                            buf.ctypes.data_as(C.POINTER(C.c_uint64)), nw.value, C.byref(nw))
t = buf.reshape(-1, 3).astype(np.int64)
t = t[t[:, 1] > 0]
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) * 10e-6, (t[:, 1] - t0) * 10e-6                      # ms
tile, itc, its = t[:, 2] & 0xFFFFFF, (t[:, 2] >> 24) & 0xFFFFF, (t[:, 2] >> 44) & 0xFFFFF
dur = en - st
span = en.max()
print(f"{cfg} chunks {FIRST}::{STEP}: {len(t)} waves, kernel span {span:.4f} ms", flush=True)
print("wave duration ms: mean %.4f  p50 %.4f  p90 %.4f  p99 %.4f  max %.4f" %
      (dur.mean(), *np.percentile(dur, [50, 90, 99]), dur.max()), flush=True)
# resident waves over time
grid = np.linspace(0, span, 201)
act = np.array([((st <= x) & (en > x)).sum() for x in grid])
peak = act.max()
for f in (0.9, 0.75, 0.5, 0.25):
    idx = np.where(act >= f * peak)[0]
    last = grid[idx[-1]] if len(idx) else 0
    print(f"resident >= {int(f*100)}% of peak ({peak}) until {last:.4f} ms ({last / span * 100:.1f}% of span)", flush=True)
print("resident waves every 5% of the span:", " ".join(str(int(a)) for a in act[::10]), flush=True)
# waves that start in the last 25% of the span and their durations
late = st > 0.75 * span
print(f"waves starting in the last 25%: {late.sum()}, mean duration {dur[late].mean() if late.any() else 0:.4f} ms", flush=True)
wpb = 1                                                 # one-wave blocks (render.hip kRenderBlock)
gx = (W + 8 * wpb - 1) // (8 * wpb)
top = np.argsort(-dur)[:10]
for k in top:
    blk = int(tile[k]); wv = int(k % wpb)
    print(f"  slow wave: tile {blk} (px x {(blk % gx) * 8 * wpb + wv * 8}, chunk {FIRST + STEP * (blk // gx)}) "
          f"start {st[k]:.4f} dur {dur[k]:.4f} ms, longest lane: {itc[k]} closest + {its[k]} any-hit iterations")
print("longest-lane iterations (closest+any-hit): p50 %d p90 %d p99 %d max %d; us per iteration of the slowest "
      "10 waves: %s" % (*np.percentile(itc + its, [50, 90, 99]), (itc + its).max(),
                         " ".join(f"{dur[k] * 1e3 / max(1, itc[k] + its[k]):.3f}" for k in top)), flush=True)
print("corr(duration, longest-lane iterations) = %.3f" % np.corrcoef(dur, itc + its)[0, 1], flush=True)
# per-chunk mean duration (image rows)
ch = tile // gx
cm = np.bincount(ch, weights=dur) / np.maximum(np.bincount(ch), 1)
print("mean wave duration per 8-row chunk (every 4th):", " ".join(f"{x:.3f}" for x in cm[::4]), flush=True)
# start time of each chunk's first wave (dispatch progress)
cs = np.array([st[ch == c].min() if (ch == c).any() else 0 for c in range(ch.max() + 1)])
print("first start per chunk (every 8th, ms):", " ".join(f"{x:.3f}" for x in cs[::8]), flush=True)
np.save(os.path.join(ROOT, "gpurun_out", f"timeline_{cfg}_{FIRST}_{STEP}_o{TAG}.npy"), t)
