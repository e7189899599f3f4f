"""Kernel time of the C3 (or C5) frame for several builds of libmyrt.so (A/B on one box).
usage: probe_lib.py c3 myraytracer_amd/libmyrt.so build_variants/libmyrt_X.so ...
Each library runs in its own subprocess (a process binds one libmyrt)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[2] == "--child":
    sys.path.insert(0, ROOT)
    import torch
    import myraytracer_amd as M
    from myraytracer_amd import scenes
    cfg = sys.argv[1]
    sc = {"c3": scenes.scene_c3, "c5": scenes.scene_c5, "c3i": scenes.scene_c3_instanced,
          "c3g": scenes.scene_c3_glass, "c2": scenes.scene_c2}[cfg](path_dir=os.path.join(ROOT, "scenes_cache"))
    eng = M.RayTracerEngine(sc)
    W, H = sc.cameras[0].image_resolution
    out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    res = []
    NS = int(os.environ.get("PROBE_N", "1"))     # N > 1: the slowest of the N C4 shares (chunks r::N)
    sel = os.environ.get("PROBE_SEL")            # "first:step": one chunk selection instead
    shares = [tuple(int(x) for x in sel.split(":"))] if sel else [(r, NS) for r in range(NS)]
    for rep in range(3):
        worst = 0.0
        for r, NS_ in shares:
            for _ in range(3):
                eng.render_device(out.data_ptr(), 0, r, NS_, stream=s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                eng.render_device(out.data_ptr(), 0, r, NS_, stream=s)
            e1.record()
            torch.cuda.synchronize()
            worst = max(worst, e0.elapsed_time(e1) / 20)
        res.append(worst)
    import hashlib
    h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
    print(f"{cfg} {sel or f'N={NS}'} {os.path.basename(os.environ['MYRT_LIB'])}: " + " ".join(f"{x:.4f}" for x in res)
          + f" ms  (min {min(res):.4f})  frame sha1 {h}", flush=True)
    sys.exit(0)
cfg = sys.argv[1]
for rnd in range(2):
    for spec in sys.argv[2:]:
        # LIB or LIB:VAR=VALUE,... (environment switches read per launch)
        lib, _, envs = spec.partition(":")
        env = dict(os.environ, MYRT_LIB=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in envs.split(",") if kv)
        if envs:
            print(f"  [{envs}]", flush=True)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), cfg, "--child"], env=env)
        if r.returncode != 0:
            sys.exit(r.returncode)
