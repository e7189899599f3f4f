"""Per-lane walk iterations of the C3 megakernel (a -DMYRT_WAVE_TIMES=2 build, MYRT_LIB): how many
wave iterations the closest-hit and any-hit phases take per 8x8 tile (its longest lane each), the
bound a merged per-lane primary->shadow loop would reach (longest lane of the sums), and the SIMD
efficiency of each."""
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
sc = scenes.scene_c3(path_dir=os.path.join(ROOT, "scenes_cache")) if cfg == "c3" else \
    scenes.scene_c5(path_dir=os.path.join(ROOT, "scenes_cache"))
eng = M.RayTracerEngine(sc)
W, H = sc.cameras[0].image_resolution
out = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
lib = M.load_library()
nw = C.c_int64()
r = lib.rt_debug_wave_times(eng.handle, 0, 0, 0, 1, C.c_void_p(out.data_ptr()), None, 0, C.byref(nw))
assert r == 0, r
torch.cuda.synchronize()
a = out.cpu().numpy()
p, s = a[..., 0], a[..., 1]
def tiles(x):
    return x.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
P, S = tiles(p), tiles(s)
mp, ms, mps = P.max(1), S.max(1), (P + S).max(1)
print(f"{cfg}: {P.shape[0]} tiles; lane iterations closest {P.sum():.0f} any-hit {S.sum():.0f}")
print(f"wave iterations: closest {mp.sum():.0f} (eff {P.sum() / 64 / mp.sum():.3f}), any-hit {ms.sum():.0f} "
      f"(eff {S.sum() / 64 / ms.sum():.3f}), two phases {mp.sum() + ms.sum():.0f}")
print(f"merged per-lane loop bound: {mps.sum():.0f} wave iterations (eff {(P + S).sum() / 64 / mps.sum():.3f}), "
      f"{(1 - mps.sum() / (mp.sum() + ms.sum())) * 100:.1f}% fewer")
# thresholded transitions: lanes done with their primary start shadows once k lanes are done
for frac in (0.25, 0.5):
    tot = 0
    for t in range(P.shape[0]):
        pp, ss = np.sort(P[t]), S[t][np.argsort(P[t])]
        # lanes finish primary in order of pp; transitions when >= frac*64 new lanes idle, or at the end
        k = max(1, int(frac * 64)); i = k - 1; start = {}; end = 0
        cut = []
        while i < 64:
            cut.append(i); i += k
        if cut[-1] != 63: cut.append(63)
        lo = 0
        for c in cut:
            tt = pp[c]                          # transition time
            for l in range(lo, c + 1):
                end = max(end, tt + ss[l])
            lo = c + 1
        tot += max(end, pp[-1])
    print(f"transition every {int(frac*64)} finished lanes: {tot:.0f} wave iterations "
          f"({(1 - tot / (mp.sum() + ms.sum())) * 100:.1f}% fewer)")
if os.environ.get("SAVE"):
    np.savez_compressed(os.environ["SAVE"], p=p.astype(np.uint16), s=s.astype(np.uint16))
