import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import myraytracer_amd as M
from myraytracer_amd import scenes
import oracle
sc = scenes.scaled(scenes.scene_c2(inline=True), 320, 240)
ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
eng = M.RayTracerEngine(sc)
for n in ["0", "1", "2", "3", "7", "15", "31"]:
    os.environ["MYRT_LDS_TOP"] = n
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    d = np.abs(rgb - ref).max(-1)
    bad = np.argwhere(d > 1e-5)
    print(n, "bad px", len(bad), "shadow", st.shadow_rays, ost.shadow_rays, "traced", st.shadow_rays_traced, ost.shadow_rays_used,
          "first bad", bad[:5].tolist(), flush=True)
