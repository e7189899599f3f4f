#!/usr/bin/env python3
"""bench.py — Mrays/s (primary+shadow) of the renderer core on MI355X.

Workload (BASELINE.json configs[2], "C3"): a ~1.02M-triangle single-mesh PLY scene
(512^2 heightfield + 24 icospheres, seeded; no Stanford bunny exists offline),
1920x1080, 1 spp, 1 point light, shadow rays on.  One "step" = one full frame of the
hot path (primary ray generation, TLAS/BLAS traversal, Moeller-Trumbore, Whitted
shading with shadow rays), FP64, scene and output resident in HBM.

N GPUs (torchrun, one process per GPU): pixels are independent (each seeds its own
PCG32), so the path shards with no collective on the data path.  Default
`--scaling weak` (the contract for a partitioned path): every rank renders one full C3
frame per step from its own scene replica - per-GPU work is fixed as N grows.
`--scaling strong` is configs[3] "C4": ONE frame, 8-row chunk c on rank c mod N.

Timed region: K frames bracketed by barrier + device sync; value = (primary + shadow
rays of all ranks) / max-over-ranks wall time.  Roofline: algorithmic
bytes B = 56 N_nodeFetch + 72 N_triTest + 72 N_smoothHit + 24 N_pixel counted in the
reference's traversal order by a counting launch (equal to the oracle's tally), divided
by the average frame time from HIP events on the launch stream; `traffic` = PMC HBM
bytes per launch from profiles/traffic_<config>.json (tools/pmc_traffic.py).
cpu_baseline: the C++ restatement of the reference CPU renderer (oracle/, test
infrastructure) on a bounded sample of the same frame, rank 0, N = 1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    p.add_argument("--scaling", default="weak", choices=["strong", "weak"],
                   help="strong: one frame tile-partitioned over ranks (C4); weak: every rank renders a full frame")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-path", action="store_true", help="skip the rt_render (host buffer) measurement")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, available cores)")
    p.add_argument("--cache", default=os.path.join(ROOT, "scenes_cache"))
    p.add_argument("--traffic-json", default="auto",
                   help="PMC traffic summary (tools/pmc_traffic.py output); auto = profiles/traffic_<config>.json")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    # MYRT_BENCH_DEVICE pins every rank to one device: rehearsing N ranks on a 1-GPU box
    dev_override = os.environ.get("MYRT_BENCH_DEVICE")
    local = int(dev_override) if dev_override is not None else local
    torch.cuda.set_device(local)

    import myraytracer_amd as M
    from myraytracer_amd import scenes

    t0 = time.time()
    if args.config == "c3":
        scene = scenes.scene_c3(path_dir=args.cache)
        workload = "C3: ~1.02M-tri PLY (heightfield+24 icospheres), 1920x1080, 1 spp, 1 point light, shadows"
    elif args.config == "c2":
        scene = scenes.scene_c2(path_dir=args.cache)
        workload = "C2: ~69k-tri PLY bunny stand-in, 800x600, 1 spp, 1 point light"
    else:
        scene = scenes.scene_c5(path_dir=args.cache)
        workload = "C5: ~10M-tri (2 meshes, mirror spheres), 3840x2160, depth-4 reflections"
    eng = M.RayTracerEngine(scene, devices=[local])
    info = eng.info()
    log(f"[rank {rank}] scene ready in {time.time() - t0:.1f}s: tris={info.triangles} recs={info.blas_nodes} "
        f"build={info.build_ms:.0f}ms upload={info.upload_ms:.0f}ms dev={info.device_bytes / 1e6:.0f}MB")

    cam = scene.cameras[0]
    W, H = cam.image_resolution
    if args.scaling == "strong" and world > 1:
        first, step = rank, world          # C4: 8-row chunks dealt round-robin to ranks
    else:
        first, step = 0, 1
    rows = M.rows_for_chunks(H, first, step)
    out = torch.empty((max(rows, 1), W, 3), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream

    def frame():
        eng.render_device(out.data_ptr(), 0, first, step, stream=sptr)

    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize()
    st = eng.collect_stats()
    n = int(max(1, cam.num_samples) ** 0.5)
    rays_primary = rows * W * n * n
    rays_shadow = int(st.shadow_rays)
    rays_secondary = int(st.secondary_rays)     # reflection rays: reported, not in `value`
    rays_rank = rays_primary + rays_shadow

    # ---- timed region: K frames, barrier + sync on both sides
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_begin = time.perf_counter()
    for k in range(args.steps):
        starts[k].record(stream)
        frame()
        ends[k].record(stream)
    torch.cuda.synchronize()
    t_elapsed = time.perf_counter() - t_begin
    if world > 1:
        dist.barrier()
    kernel_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends)) / args.steps

    t_max = t_elapsed
    rays_total = rays_rank * args.steps
    if world > 1:
        tt = torch.tensor([t_elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        rr = torch.tensor([rays_total], dtype=torch.float64)
        dist.all_reduce(rr, op=dist.ReduceOp.SUM)
        rays_total = float(rr.item())
    value = rays_total / t_max / 1e6
    ms_per_step = t_max * 1e3 / args.steps

    # ---- roofline: algorithmic bytes of one launch, counted on the GPU in
    # the reference's traversal order (rt_render_device_counted; equal to the oracle's tally,
    # tests/test_gpu_parity.py), divided by the average launch time of the timed frames.
    wc = eng.work_counters(out.data_ptr(), 0, first, step, stream=sptr)
    alg_bytes = (56 * wc.ref_node_fetches + 72 * wc.ref_tri_tests + 72 * wc.ref_smooth_hits
                 + 24 * wc.ref_pixels)
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic, tpath = None, args.traffic_json
    if tpath == "auto":
        tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if tpath and os.path.exists(tpath) and world == 1:
        try:
            with open(tpath) as fh:
                traffic = json.load(fh).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": os.path.relpath(tpath, ROOT) if traffic is not None else None,
                "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": int(alg_bytes),
                "alg_bytes_per_ray": round(alg_bytes / max(1, rays_rank), 1),
                "alg_counts": {"node_fetches": int(wc.ref_node_fetches), "tri_tests": int(wc.ref_tri_tests),
                               "smooth_hits": int(wc.ref_smooth_hits), "pixels": int(wc.ref_pixels)},
                "simd_efficiency": {
                    "closest": round(wc.lane_steps_closest / max(1, 64 * wc.wave_steps_closest), 3),
                    "shadow": round(wc.lane_steps_shadow / max(1, 64 * wc.wave_steps_shadow), 3)},
                "executed": {"records_128B": int(wc.records_fetched), "tri_tests": int(wc.tri_tests),
                             "normal_fetches": int(wc.normal_fetches), "pixels": int(wc.pixels),
                             "load_bytes": int(128 * wc.records_fetched + 80 * wc.tri_tests
                                               + 72 * wc.normal_fetches + 24 * wc.pixels)}}

    # ---- host-buffer path (rt_render: render + D2H of the FP64 framebuffer + host scatter,
    # batches overlapped with the copies).  Reported next to `value`, never as `value`.
    host_path = None
    if not args.no_host_path:
        try:
            import numpy as np
            host_buf = np.zeros((rows, W, 3), dtype=np.float64)        # caller-owned, reused
            eng.render_rows(0, first, step, False, out=host_buf)        # staging warm-up
            t_h = time.perf_counter()
            nh = 5
            for _ in range(nh):
                eng.render_rows(0, first, step, False, out=host_buf)
            ms_h = (time.perf_counter() - t_h) * 1e3 / nh
            host_path = {"ms_per_frame": round(ms_h, 4), "value": round(rays_rank / (ms_h * 1e-3) / 1e6, 2),
                         "unit": "Mrays/s", "what": "rt_render wall time incl. D2H of the FP64 RGB framebuffer"}
            # caller buffer in page-locked memory (rt_host_alloc): rows DMA'd straight into it
            pin_rgb, _ = eng.alloc_frame(0, first, step, rgba=False)
            eng.render_rows(0, first, step, False, out=pin_rgb)
            t_h = time.perf_counter()
            for _ in range(nh):
                eng.render_rows(0, first, step, False, out=pin_rgb)
            ms_p = (time.perf_counter() - t_h) * 1e3 / nh
            host_path["pinned"] = {"ms_per_frame": round(ms_p, 4), "value": round(rays_rank / (ms_p * 1e-3) / 1e6, 2),
                                   "what": "same into a page-locked caller buffer (rt_host_alloc): the kernel stores rows into it over PCIe, no copy"}
            del pin_rgb
        except Exception as e:  # pragma: no cover
            log("host path failed:", e)

    # ---- CPU baseline (rank 0, N = 1 only): oracle on a bounded sample of the same frame
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(scene, H, args)
        except Exception as e:  # pragma: no cover
            log("cpu baseline failed:", e)
            cpu = {"value": None, "unit": "Mrays/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}

    if rank == 0:
        line = {
            "metric": "Mrays/s (primary+shadow), 1920x1080 / 1M-tri PLY, at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if args.scaling == "strong" else "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (seeded scene generator; no bunny/assets offline)",
            "config": {"workload": workload, "width": W, "height": H, "spp": max(1, cam.num_samples),
                       "triangles": int(info.triangles),
                       "partition": (f"8-row chunks round-robin over {world} GPU(s)" if args.scaling == "strong"
                                     else f"one full frame per GPU per step, {world} GPU(s), no collective"),
                       "rays_per_frame": int(rays_rank) if world == 1 else None,
                       "secondary_rays_per_frame": rays_secondary if world == 1 else None},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "host_path": host_path,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(scene, H, args):
    """Oracle (C++ restatement of the reference CPU renderer) on every k-th 8-row chunk."""
    import oracle
    cores = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
    t0 = time.time()
    o = oracle.OracleScene(scene if scene.objects[0].ply_path is None else _inline(scene))
    build_s = time.time() - t0
    nchunks = (H + 7) // 8
    # calibrate on one chunk, then size the sample to ~cpu_seconds of wall time: a strided
    # subset of the frame's 8-row chunks, or whole frames repeated when one frame is shorter
    _, st = o.render(0, nchunks // 2, nchunks, threads=1)
    per_chunk_s = max(st.milliseconds / 1e3, 1e-4)
    want = max(1, int(args.cpu_seconds * cores / per_chunk_s))
    stride = max(1, nchunks // want)
    frames = max(1, min(50, int(want // nchunks))) if stride == 1 else 1
    rays = 0
    ms = 0.0
    px = 0
    for _ in range(frames):
        _, st = o.render(0, 0, stride, threads=cores)
        rays += st.primary_rays + st.shadow_rays
        ms += st.milliseconds
        px += st.pixels
    what = (f"{frames} full frame(s)" if stride == 1 else f"every {stride}th 8-row chunk of the frame")
    return {"value": round(rays / (ms / 1e3) / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"{what} ({px} px, {rays} rays, {ms / 1e3:.1f}s on {cores} threads; "
                      f"oracle BVH build {build_s:.1f}s excluded)"}


def _inline(scene):
    """The oracle takes inline arrays: read the PLY paths with the product's loader."""
    import copy
    import myraytracer_amd as M
    s = copy.deepcopy(scene)
    for obj in s.objects:
        if isinstance(obj, M.Mesh) and obj.ply_path is not None:
            m = M.ply_load(obj.ply_path)
            obj.positions, obj.indices = m["positions"], m["indices"]
            obj.normals = m["normals"]
            obj.indices_one_based = False
            obj.ply_path = None
    return s


if __name__ == "__main__":
    main()
