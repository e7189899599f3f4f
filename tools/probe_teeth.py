"""Teeth of the transformed walks' widening on one library build (MYRT_LIB): the far-instance
near-vertex ray set of tests/test_gpu_wide_bound.py, closest-hit mismatches against the oracle at
wide_delta_scale 0 and 1000, for option fit = 1 (flattened instance tree) and 0 (tw_walk).

usage: MYRT_LIB=... python tools/probe_teeth.py   (GPU box; prints one line per setting)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import myraytracer_amd as M  # noqa: E402
import oracle  # noqa: E402
import test_gpu_wide_bound as W  # noqa: E402


def main():
    sc, mats, centre = W._far_instances()
    mesh = sc.objects[0]
    P, F = np.asarray(mesh.positions), np.asarray(mesh.indices)
    rng = np.random.RandomState(91)
    Os, Ds = [], []
    for M4 in mats:
        Pw = P @ M4[:3, :3].T + M4[:3, 3]
        O, D = W._near_vertex_rays(Pw, F, 5000, rng, 4.0e4)
        Os.append(O); Ds.append(D)
    O, D = np.concatenate(Os), np.concatenate(Ds)
    to, po, no, mo = oracle.OracleScene(sc).trace_rays(O, D)
    lib = M.load_library()
    for fit in (1, 0):
        for permille in (0, 1000):
            eng = M.RayTracerEngine(sc)
            if hasattr(lib, "rt_scene_set_unsafe_option"):
                eng.set_unsafe_option("wide_delta_scale", permille)
            else:
                eng.set_option("wide_delta_scale", permille)
            try:
                eng.set_option("fit", fit)
            except Exception:
                if fit:
                    eng.close()
                    continue
            tg, pg, ng, mg = eng.trace_rays(O, D)
            eng.close()
            bad = (tg.view(np.uint64) != to.view(np.uint64)) | (mg != mo)
            hit = np.isfinite(to) & np.isfinite(tg)
            bad |= hit & ((pg != po).any(1) | (ng != no).any(1))
            print(f"lib={os.path.basename(os.environ.get('MYRT_LIB', 'libmyrt.so'))} fit={fit} permille={permille}: "
                  f"{int(bad.sum())} / {len(O)} closest hits differ", flush=True)


if __name__ == "__main__":
    main()
