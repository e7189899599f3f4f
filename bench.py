#!/usr/bin/env python3
"""bench.py — Mrays/s (primary+shadow) of the renderer core on MI355X.

Workload (BASELINE.json configs[2], "C3"): a ~1.02M-triangle single-mesh PLY scene
(512^2 heightfield + 24 icospheres, seeded; no Stanford bunny exists offline),
1920x1080, 1 spp, 1 point light, shadow rays on, FP64 throughout.

One "step" = one frame through the public render path, timed as SURVEY.md §8(d) defines
it: render wall time with the scene resident in HBM, INCLUDING the device->host delivery
of the image and the host gather.  The image is what the reference's public
`RayTracerEngine.render` returns - RGBA8 (RayTracer.swift:115-131, 166-203: its render
time spans Renderer.render + the RGBA8 conversion).  The kernels store the RGBA8 rows
straight into a page-locked host framebuffer (host-mapped, over PCIe).  The reference's
render is `async`; frames go through rt_render_submit / rt_render_wait with `--in-flight`
(default RT_MAX_IN_FLIGHT = 16) renders in flight on 32 hardware queues, frame k into
framebuffer k mod Q, so the next frame's tiles
fill the compute units the previous frame's slowest tiles leave idle; value = K frames
delivered / wall time.  `timing.submit_to_done_ms` is one frame's latency.  Side fields
time the FP64 [Vec3] framebuffer delivered synchronously (`fp64_path`, rt_render) and the
device-only launch (`device_only`).

N GPUs: one process per GPU (torchrun; `python bench.py --gpus N` starts torchrun itself
before anything touches a GPU).  Default for N>1 is configs[3] "C4", STRONG scaling: ONE
C3 frame per step, 8-row chunk c rendered by rank c mod N (Object+Extension.swift:75-82),
every rank storing its rows into one shared page-locked framebuffer (POSIX shared memory
registered with rt_host_register) - the host-side gather, with no collective on the data
path.  `--scaling weak` (opt-in) gives every rank a full frame of its own.

value = (primary rays + shadow rays actually traversed, all ranks) / max-over-ranks wall
time of K steps bracketed by barrier + device sync.  Shadow rays whose walk is skipped
(N.L <= 0: the reference discards their result, Object+Extension.swift:123-141) are
reported apart (`rays.shadow_cast`), never in `value`.

roofline (dominant kernel = the render megakernel - for C5 the compacted bounce render's chain of
launches per frame - average duration from HIP events on its stream, taken inside rt_render): `achieved` = measured HBM bytes per launch (PMC
FETCH_SIZE x2 + WRITE_SIZE, profiles/roofline_<config>.json, same build) / kernel time,
against the 8 TB/s HBM peak.  The kernel is not HBM-bound (its working set sits in L2 and
the 256 MB Infinity Cache): `roofline.binding` names the resource that binds it (FP64 VALU
issue at ~half lane utilisation, then the vector-memory data path; from the same profile),
`roofline.pipelined` divides the same bytes by the GPU time a pipelined frame costs (the union
of the render launches in the bench's own loop under rocprofv3, profiles/overlap_<config>.json)
and `roofline.reference_work` holds the SURVEY §8(d) algorithmic bytes of the reference's
unpruned walk, counted on the GPU.
cpu_baseline: the C++ restatement of the reference CPU renderer (oracle/, test
infrastructure), rank 0, N = 1: median over whole frames at the box's CPU share, plus the
1-thread rate on a sampled subset of chunks.
"""
from __future__ import annotations

import argparse
import collections
import hashlib
import json
import mmap
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 2000 C3 frames = ~1.3 s timed at N = 1: long enough for an outside GPU-busy sampler
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--config", default="c3", choices=["c2", "c3", "c5", "c3i", "c3g", "c3d", "c3r"],
                   help="c3 (default, BASELINE configs[2]); c2 / c5 (configs[1] / [4]); c3i: C3 as 25 mesh "
                        "instances with transforms (literal TLAS->BLAS walk); c3g: C3 with glass spheres and two "
                        "area lights (full trace() kernels); c3d: the glass spheres with the point light only; c3r: c3g "
                        "with rough glass (the depth-first k_events pass)")
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                   help="strong (default): one frame per step split over the ranks (C4); "
                        "weak: every rank renders a full frame per step")
    p.add_argument("--gather", default="shared", choices=["shared", "staged"],
                   help="N > 1 strong: shared (default) = every rank's kernels store their rows straight into "
                        "one shared page-locked framebuffer; staged = rows delivered by each GPU's DMA engine "
                        "into a private page-locked frame, then copied by the rank's host thread into the "
                        "shared frame (no concurrent PCIe stores from 8 GPUs into one segment)")
    p.add_argument("--numa-placement", default="none", choices=["none", "first-touch"],
                   help="N > 1 strong, shared gather: first-touch = each rank binds its CPU affinity to its GPU's "
                        "NUMA node (when the process may run there) and touches its own rows of every shared "
                        "frame before any rank registers it, so those pages live on its GPU's socket; none = "
                        "pages land where the first registering process faults them")
    p.add_argument("--in-flight", type=int, default=0,
                   help="renders in flight (rt_render_submit); 1 = one frame at a time; 0 = RT_MAX_IN_FLIGHT (16)")
    p.add_argument("--hw-queues", type=int, default=-1,
                   help="GPU_MAX_HW_QUEUES for this process (-1 = 32: one per render in flight and the "
                        "library's own streams; 0 = HIP's default)")
    p.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                   help="render option for the run (rt_scene_set_option, INTEGRATION.md table); repeatable")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-side-paths", action="store_true", help="skip the fp64 / device-only side measurements")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = the CPU share (OMP_NUM_THREADS / affinity)")
    p.add_argument("--cpu-frames", type=int, default=3)
    p.add_argument("--cache", default=os.path.join(ROOT, "scenes_cache"))
    p.add_argument("--profile-json", default="auto",
                   help="PMC summary (tools/pmc_roofline.py); auto = profiles/roofline_<config>.json")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def relaunch_under_torchrun(args) -> int:
    """`bench.py --gpus N` outside torchrun: start one process per GPU as a child (before any
    GPU call in this process) and return its exit code."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("[bench] starting", " ".join(cmd))
    return subprocess.call(cmd)


class SharedFrame:
    """One host framebuffer shared by every rank (POSIX shared memory), page-locked in each
    process with rt_host_register so the kernels of every GPU store their rows into it."""

    def __init__(self, nbytes, rank, world, dist, tag):
        import numpy as np
        run = os.environ.get("TORCHELASTIC_RUN_ID", "") + os.environ.get("MASTER_PORT", "")
        self.path = f"/dev/shm/myrt_bench_{tag}_{hashlib.sha256(run.encode()).hexdigest()[:12]}"
        self.rank, self.world = rank, world
        if rank == 0:
            with open(self.path, "wb") as fh:
                fh.truncate(nbytes)
        if world > 1:
            dist.barrier()
        self._fh = open(self.path, "r+b")
        self._mm = mmap.mmap(self._fh.fileno(), nbytes)
        self.array = np.frombuffer(self._mm, dtype=np.uint8)   # zero-filled by the truncate

    def close(self, dist, registered=True):
        import myraytracer_amd as M
        if registered:
            M.unregister_host(self.array)  # the mapping itself goes with the process
        if self.world > 1:
            dist.barrier()
        if self.rank == 0:
            os.unlink(self.path)


def _cpulist(text):
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def _ranges(cpus):
    cpus = sorted(cpus)
    out, k = [], 0
    while k < len(cpus):
        j = k
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(f"{cpus[k]}-{cpus[j]}" if j > k else str(cpus[k]))
        k = j + 1
    return ",".join(out)


def numa_nodes():
    """{node: [cpus]} from sysfs (empty when the machine exposes no NUMA topology)."""
    base = "/sys/devices/system/node"
    nodes = {}
    try:
        for d in os.listdir(base):
            if d.startswith("node") and d[4:].isdigit():
                with open(os.path.join(base, d, "cpulist")) as fh:
                    nodes[int(d[4:])] = _cpulist(fh.read())
    except OSError:
        pass
    return nodes


def gpu_numa_node(dev):
    """NUMA node of GPU `dev` (its PCI function's numa_node in sysfs), or None."""
    import torch
    try:
        pr = torch.cuda.get_device_properties(dev)
        dom, bus, slot = (int(getattr(pr, "pci_domain_id", 0)), int(getattr(pr, "pci_bus_id")),
                          int(getattr(pr, "pci_device_id")))
        path = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{slot:02x}.0/numa_node"
        with open(path) as fh:
            n = int(fh.read().strip())
        return {"node": n if n >= 0 else None, "pci": f"{dom:04x}:{bus:02x}:{slot:02x}.0"}
    except Exception as e:  # pragma: no cover - depends on the machine
        return {"node": None, "error": f"{type(e).__name__}: {e}"}


def pages_by_node(addr, nbytes):
    """{node: pages} of the pages in [addr, addr + nbytes) that are present (move_pages(2) with no
    target nodes reports each page's node; x86-64 syscall 279).  None where unavailable."""
    import ctypes
    if nbytes <= 0:
        return {}
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        pg = os.sysconf("SC_PAGE_SIZE")
        first = addr // pg * pg
        n = (addr + nbytes - first + pg - 1) // pg
        pages = (ctypes.c_void_p * n)(*[first + k * pg for k in range(n)])
        status = (ctypes.c_int * n)()
        if libc.syscall(279, 0, ctypes.c_ulong(n), pages, None, status, 0) != 0:
            return None
    except Exception:  # pragma: no cover - depends on the machine
        return None
    out = collections.Counter(int(x) for x in status if x >= 0)
    return {str(k): v for k, v in sorted(out.items())}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_under_torchrun(args))
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # renders in flight overlap only on hardware queues of their own: HIP's default of 4 queues
    # per process is shared by the library's streams (tools/probe_submit.py: a C4/8 share takes
    # 0.155 / 0.12 / 0.095 ms per frame with 4 / 8 / 16 queues and 8 in flight;
    # tools/probe_shares.py: 0.086 ms with 32 queues and 16 in flight, the whole C3 frame
    # 0.642 ms).  Set before anything initialises HIP.
    if args.in_flight <= 0:
        args.in_flight = 16
    if args.hw_queues < 0:
        # ranks rehearsed on one GPU (MYRT_BENCH_DEVICE) share its hardware queue slots: more
        # than 32 queues on one GPU time-slice (2 ranks x 32: 10.6 ms per frame instead of 0.35)
        args.hw_queues = 32 // (world if "MYRT_BENCH_DEVICE" in os.environ else 1)
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))

    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # barriers + scalar reductions only; gloo announces its connections on stdout, which is
        # kept for the one JSON line: send that chatter to stderr while the group forms
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", init_method="env://")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    # MYRT_BENCH_DEVICE pins every rank to one device: rehearsing N ranks on a 1-GPU box
    dev_override = os.environ.get("MYRT_BENCH_DEVICE")
    local = int(dev_override) if dev_override is not None else local
    torch.cuda.set_device(local)
    # NUMA: this rank's GPU node, CPU affinity, and (opt-in) the affinity bound to the GPU's node
    nodes = numa_nodes()
    gnode = gpu_numa_node(local)
    numa = {"gpu": gnode, "placement": args.numa_placement, "affinity_before": _ranges(os.sched_getaffinity(0))}
    if args.numa_placement == "first-touch" and gnode.get("node") is not None and gnode["node"] in nodes:
        want = set(nodes[gnode["node"]]) & os.sched_getaffinity(0)
        if want:
            os.sched_setaffinity(0, want)
        numa["bound_to_gpu_node"] = bool(want)
    aff = os.sched_getaffinity(0)
    numa["affinity"] = _ranges(aff)
    numa["affinity_nodes"] = sorted(n for n, c in nodes.items() if aff & set(c))

    import myraytracer_amd as M
    from myraytracer_amd import _abi as A
    from myraytracer_amd import scenes

    t0 = time.time()
    if args.config == "c3":
        scene = scenes.scene_c3(path_dir=args.cache)
        workload = "C3: ~1.02M-tri PLY (heightfield+24 icospheres), 1920x1080, 1 spp, 1 point light, shadows"
    elif args.config == "c2":
        scene = scenes.scene_c2(path_dir=args.cache)
        workload = "C2: ~69k-tri PLY bunny stand-in, 800x600, 1 spp, 1 point light"
    elif args.config == "c3i":
        scene = scenes.scene_c3_instanced(path_dir=args.cache)
        workload = ("C3i: C3's geometry as 25 mesh instances with non-identity transforms (terrain + 24 instances "
                    "of one icosphere BLAS), 1920x1080, 1 spp, 1 point light, shadows: the literal TLAS->BLAS walk")
    elif args.config == "c3d":
        scene = scenes.scene_c3_glass(path_dir=args.cache, area_lights=False)
        workload = ("C3d: C3's geometry with 24 glass (dielectric, Beer) spheres, 1 point light, "
                    "1920x1080, 1 spp, maxRecursionDepth 4: level passes + node shading + render_full")
    elif args.config == "c3r":
        scene = scenes.scene_c3_glass(path_dir=args.cache, rough=True)
        workload = ("C3r: C3g with rough glass (roughness 0.05), 1 point + 2 area lights, 1920x1080, 1 spp, "
                    "maxRecursionDepth 4: depth-first k_events + k_jscan + render_full")
    elif args.config == "c3g":
        scene = scenes.scene_c3_glass(path_dir=args.cache)
        workload = ("C3g: C3's geometry with 24 glass (dielectric, Beer) spheres, 1 point + 2 area lights, "
                    "1920x1080, 1 spp, maxRecursionDepth 4: full trace() kernels")
    else:
        scene = scenes.scene_c5(path_dir=args.cache)
        workload = "C5: ~10M-tri (2 meshes, mirror spheres), 3840x2160, depth-4 reflections"
    eng = M.RayTracerEngine(scene, devices=[local])
    options = {}
    for o in args.option:
        name, _, value = o.partition("=")
        eng.set_option(name, int(value))
        options[name] = int(value)
    info = eng.info()
    log(f"[rank {rank}] scene ready in {time.time() - t0:.1f}s: tris={info.triangles} recs={info.blas_nodes} "
        f"build={info.build_ms:.0f}ms upload={info.upload_ms:.0f}ms dev={info.device_bytes / 1e6:.0f}MB")

    cam = scene.cameras[0]
    W, H = cam.image_resolution
    strong = args.scaling == "strong"
    first, step = (rank, world) if strong else (0, 1)
    rows = M.rows_for_chunks(H, first, step)
    n = int(max(1, cam.num_samples) ** 0.5)

    # ---- the framebuffers the images are delivered into (RGBA8, whole frame, row 0 = top): one
    # per render in flight; frame k goes to framebuffer k mod Q
    Q = max(1, min(args.in_flight, A.RT_MAX_IN_FLIGHT))
    shared = []
    staged = strong and world > 1 and args.gather == "staged"
    my_rows = None
    if strong and world > 1:
        for q in range(Q):
            sf = SharedFrame(W * H * 4, rank, world, dist, f"{args.config}{q}")
            shared.append(sf)
        if args.numa_placement == "first-touch" and not staged:
            # every rank first-touches its own rows (8-row chunks c = rank mod world) while bound to
            # its GPU's node; registration (which faults every page it touches first) waits for all
            mine_rows = np.concatenate([np.arange(8 * c, min(8 * c + 8, H))
                                        for c in range(first, (H + 7) // 8, step)] or [np.empty(0, np.int64)])
            for sf in shared:
                sf.array.reshape(H, W, 4)[mine_rows] = 0
            dist.barrier()
        if not staged:
            for sf in shared:
                M.register_host(sf.array)
        gathered = [sf.array.reshape(H, W, 4) for sf in shared]
        if staged:
            # private page-locked frames, written by the DMA engine; the host copies this rank's
            # rows into the shared frame after each wait (8-row chunks c = rank mod world)
            fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]
            for fb_ in fbs:
                fb_[:] = 0
            my_rows = np.concatenate([np.arange(8 * c, min(8 * c + 8, H))
                                      for c in range(first, (H + 7) // 8, step)] or [np.empty(0, np.int64)])
            eng.set_option("submit_dma", 1)
        else:
            fbs = gathered
    else:
        fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]
        for fb_ in fbs:
            fb_[:] = 0
        gathered = fbs

    # frames through rt_render_submit / rt_render_wait with Q renders in flight (the reference's
    # render is async, RayTracer.swift:137-205), arguments marshalled once (engine.frame_pipeline)
    submit, wait = eng.frame_pipeline(0, first, step, fbs, frame_layout=True)
    if my_rows is not None:                           # frame_pipeline rendered every buffer once
        for q in range(Q):
            gathered[q][my_rows] = fbs[q][my_rows]

    submit_s = [0.0]                                  # host time inside rt_render_submit (timed frames)

    def finish(k, ticket, stats_out):
        s_ = wait(ticket)
        if my_rows is not None:                       # staged gather: this rank's rows to the shared frame
            gathered[k % Q][my_rows] = fbs[k % Q][my_rows]
        if stats_out is not None:
            stats_out.append((s_.kernel_ms, s_.milliseconds))
        return s_

    def run(k_frames, stats_out=None):
        pend = collections.deque()
        for k in range(k_frames):
            if len(pend) == Q:
                finish(*pend.popleft(), stats_out)
            if stats_out is not None:
                ts = time.perf_counter()
                pend.append((k, submit(k)))
                submit_s[0] += time.perf_counter() - ts
            else:
                pend.append((k, submit(k)))
        last = None
        while pend:
            last = finish(*pend.popleft(), stats_out)
        return last

    st = run(max(1, args.warmup))
    scratch_after_warmup = int(eng.info().scratch_bytes)
    # where this rank's rows of the delivered frames live (pages per NUMA node; the shared frames
    # for N > 1, this rank's own page-locked frames for N = 1)
    if strong and world > 1 and not staged:
        pg = collections.Counter()
        row_b = W * 4
        for sf in shared:
            base = sf.array.ctypes.data
            for c in range(first, (H + 7) // 8, step):
                got = pages_by_node(base + 8 * c * row_b, min(8, H - 8 * c) * row_b) or {}
                for k_, v_ in got.items():
                    pg[k_] += v_
        numa["frame_pages_by_node"] = dict(pg)
        numa["frame_pages_what"] = "this rank's rows of the shared frames: pages per NUMA node (move_pages)"
    else:
        pg = collections.Counter()
        for fb_ in fbs:
            for k_, v_ in (pages_by_node(fb_.ctypes.data, fb_.nbytes) or {}).items():
                pg[k_] += v_
        numa["frame_pages_by_node"] = dict(pg)
        numa["frame_pages_what"] = "this rank's page-locked frames: pages per NUMA node (move_pages)"
    rays_primary = rows * W * n * n
    shadow_cast, shadow_traced = int(st.shadow_rays), int(st.shadow_rays_traced)
    rays_rank = rays_primary + shadow_traced

    # ---- timed region: K frames, barrier + sync on both sides
    per = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_begin = time.perf_counter()
    run(args.steps, per)
    torch.cuda.synchronize()
    t_elapsed = time.perf_counter() - t_begin
    calls = [b for _, b in per]
    if world > 1:
        dist.barrier()
    # the render kernel's own launch duration (roofline): HIP events around it, one frame at a
    # time (with frames in flight the event span also covers the overlapped neighbours)
    one = eng.frame_renderer(0, first, step, rgb=None, rgba=fbs[0], frame_layout=True)
    sync = []
    for _ in range(max(5, min(args.steps, 20))):
        s_ = one()
        sync.append((s_.kernel_ms, s_.milliseconds))
    kernel_ms = statistics.mean(a for a, _ in sync)
    sync_ms = statistics.mean(b for _, b in sync)

    t_max = t_elapsed
    tot = np.array([rays_rank, rays_primary + shadow_cast, shadow_cast, shadow_traced], dtype=np.float64) * args.steps
    per_rank = None
    if world > 1:
        # the same pipelined loop with the image left in HBM (option submit_dma = 2: rows rendered
        # into device staging, not delivered): each rank's device-only time per frame, so the first
        # multi-GPU line tells compute scaling from host-gather bandwidth
        dma_prev = eng.get_option("submit_dma")
        eng.set_option("submit_dma", 2)
        n_dev = max(20, min(args.steps, 200))
        torch.cuda.synchronize()
        td = time.perf_counter()
        saved = my_rows
        my_rows = None
        run(n_dev)
        my_rows = saved
        torch.cuda.synchronize()
        dev_ms = (time.perf_counter() - td) * 1e3 / n_dev
        eng.set_option("submit_dma", dma_prev)
        # every rank's own clock and host submit cost, so an N > 1 line shows its imbalance
        mine = torch.tensor([t_elapsed * 1e3 / args.steps, submit_s[0] * 1e6 / args.steps, float(rows), dev_ms],
                            dtype=torch.float64)
        allr = [torch.zeros(4, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(allr, mine)
        numa_r = [None] * world
        dist.all_gather_object(numa_r, numa)
        ms_r = [round(float(x[0]), 4) for x in allr]
        dv_r = [round(float(x[3]), 4) for x in allr]
        per_rank = {"ms_per_step": ms_r, "device_ms_per_frame": dv_r,
                    "submit_us_per_frame": [round(float(x[1]), 2) for x in allr],
                    "rows": [int(x[2]) for x in allr], "min_ms": min(ms_r), "max_ms": max(ms_r),
                    "device_max_ms": max(dv_r), "delivery_overhead": round(max(ms_r) / max(1e-9, max(dv_r)), 4),
                    "imbalance": round(max(ms_r) / max(1e-9, min(ms_r)), 4), "gather": args.gather,
                    "numa": numa_r,
                    "what": "per rank: its own timed-region clock per frame (value uses the max, image delivered "
                            "to the shared host frame), the same pipelined loop with the image left in HBM "
                            f"({n_dev} frames, device_ms_per_frame), host time inside rt_render_submit per "
                            "frame, rows of the frame it renders; delivery_overhead = max delivered / max "
                            "device-only"}
    if world > 1:
        tt = torch.tensor([t_elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        rr = torch.tensor(tot)
        dist.all_reduce(rr, op=dist.ReduceOp.SUM)
        tot = rr.numpy()
        km = torch.tensor([kernel_ms], dtype=torch.float64)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_ms = float(km.item())
    value = tot[0] / t_max / 1e6
    ms_per_step = t_max * 1e3 / args.steps

    # ---- the gathered image: every row delivered (alpha 255 everywhere), and its hash (equal
    # for every N: the multi-GPU split changes nothing in the image)
    if world > 1:
        dist.barrier()
    gather = None
    if rank == 0:
        fb = gathered[(args.steps - 1) % Q]                  # the last frame delivered
        gather = {"rows_complete": bool(all(np.all(f_[:, :, 3] == 255) for f_ in gathered)),
                  "rgba8_sha256": hashlib.sha256(np.ascontiguousarray(fb).tobytes()).hexdigest(),
                  "frames_identical": bool(all(np.array_equal(f_, fb) for f_ in gathered)),
                  "mode": args.gather if (strong and world > 1) else "single"}

    # ---- roofline (profiles/roofline_<config>.json: PMC passes of this build, tools/pmc_roofline.py)
    roofline = roofline_fields(args, eng, local, first, step, rows, W, kernel_ms, rays_rank, world)

    # ---- side paths on this rank's share: FP64 framebuffer delivery, device-only launch
    side = None
    if not args.no_side_paths:
        side = side_paths(eng, first, step, rows, W, H, rays_rank, args)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(scene, H, args)
        except Exception as e:  # pragma: no cover
            log("cpu baseline failed:", e)
            cpu = {"value": None, "unit": "Mrays/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}

    for sf in shared:
        sf.close(dist, registered=not staged)
    if rank == 0:
        line = {
            "metric": "Mrays/s (primary+shadow), 1920x1080 / 1M-tri PLY, at 1/2/4/8 MI355X",
            "value": round(float(value), 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (seeded scene generator; no bunny/assets offline)",
            "config": {"workload": workload, "width": W, "height": H, "spp": max(1, cam.num_samples),
                       "triangles": int(info.triangles),
                       "partition": (f"one frame per step, 8-row chunks round-robin over {world} GPU(s), "
                                     "rows stored into shared page-locked framebuffers" if strong else
                                     f"one full frame per GPU per step, {world} GPU(s), no collective"),
                       "delivered": "RGBA8 frame in page-locked host memory (RayTracerEngine.render's image)",
                       "in_flight": Q, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "HIP default"),
                       "render_options": options},
            "rays": {"per_step": int(tot[0] / args.steps), "primary_per_step": int(rays_primary) if world == 1 else None,
                     "shadow_traced_per_step": int(tot[3] / args.steps),
                     "shadow_cast_per_step": int(tot[2] / args.steps),
                     "value_reference_count": round(float(tot[1] / t_max / 1e6), 2),
                     "note": "value counts shadow rays actually traversed; shadow_cast adds the rays the "
                             "reference casts where N.L <= 0 and discards (value_reference_count)",
                     "secondary_per_step": int(st.secondary_rays) if world == 1 else None,
                     "rewalked_per_step": int(getattr(st, "rewalked", 0)),
                     "rewalked_what": "closest-hit rays of rank 0's share that the four-wide walk handed to the "
                                      "reference-order walk (two candidates at the final t, wide.h)"},
            "per_rank": per_rank,
            "numa": numa if world == 1 else {"placement": args.numa_placement, "per_rank": "per_rank.numa"},
            "scene": {"device_bytes": int(info.device_bytes), "scratch_bytes_after_warmup": scratch_after_warmup,
                      "build_ms": round(float(info.build_ms), 1), "upload_ms": round(float(info.upload_ms), 1)},
            "timing": {"in_flight": Q, "submit_to_done_ms": round(statistics.mean(calls), 4),
                       "submit_us_per_frame": round(submit_s[0] * 1e6 / args.steps, 2),
                       "one_frame_ms": round(sync_ms, 4), "kernel_ms": round(kernel_ms, 4),
                       "what": "frames pipelined with in_flight renders submitted (rt_render_submit) before the "
                               "oldest is waited for (rt_render_wait); submit_to_done_ms = a pipelined frame's "
                               "latency from submit to image complete in host memory; one_frame_ms = the same for "
                               "one frame at a time (rt_render_ex, RenderStats.milliseconds); kernel_ms = HIP events "
                               "around the render launch in those single frames"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "gather": gather,
            "side_paths": side,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def roofline_fields(args, eng, dev, first, step, rows, W, kernel_ms, rays_rank, world):
    import torch
    out = torch.empty((max(rows, 1), W, 3), dtype=torch.float64, device=f"cuda:{dev}")
    wc = eng.work_counters(out.data_ptr(), 0, first, step, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del out
    alg_bytes = (56 * wc.ref_node_fetches + 72 * wc.ref_tri_tests + 72 * wc.ref_smooth_hits + 24 * wc.ref_pixels)
    load_bytes = 128 * wc.records_fetched + 80 * wc.tri_tests + 72 * wc.normal_fetches + 24 * wc.pixels
    prof, ppath = None, args.profile_json
    if ppath == "auto":
        ppath = os.path.join(ROOT, "profiles", f"roofline_{args.config}.json")
    if ppath and os.path.exists(ppath):
        with open(ppath) as fh:
            prof = json.load(fh)
    lib_sha = _lib_sha()
    r = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None,
         "kernel_ms": round(kernel_ms, 4),
         "kernel_ms_source": "HIP events around the render launch on its stream, inside rt_render, one frame "
                             "at a time after the timed steps"}
    if prof is not None and world == 1:
        traffic = prof["hbm_bytes_per_launch"]
        r["traffic_source"] = os.path.relpath(ppath, ROOT)
        r["profiled_kernels"] = prof.get("kernel")
        if prof.get("frame_chain"):
            # C5's compacted bounce render: a frame is a chain of launches; traffic and the
            # compute figures are per frame over the chain (tools/pmc_roofline.py), kernel_ms the
            # HIP events around the whole chain
            r["frame_chain"] = prof.get("chain")
        r["profile_build_matches"] = prof.get("lib_sha256_16") == lib_sha
        if r["profile_build_matches"]:
            # figures from another build's profile would describe that build: only a profile of
            # this very library fills achieved / frac / traffic
            r["traffic"] = int(traffic)
            r["achieved"] = round(traffic / (kernel_ms * 1e-3) / 1e9, 2)
            r["frac"] = round(r["achieved"] / HBM_PEAK_GBS, 4)
        if "lane_throughput_frac" in prof and r["profile_build_matches"]:
            # the resource that binds the kernel: VALU issue.  Every figure from ONE rocprofv3 pass
            # (tools/pmc_roofline.py --valu): busy = issue cycles / cycles, lane util = active lanes /
            # 64 per issued instruction, their product = fraction of the SIMDs' lane-cycles used
            r["compute"] = {
                "bound": "valu-issue", "valu_busy": prof["valu_busy"], "valu_lane_util": prof["valu_lane_util"],
                "lane_throughput_frac": prof["lane_throughput_frac"],
                "valu_insts_per_launch": prof.get("valu_insts_per_launch"),
                "source": os.path.relpath(ppath, ROOT) + " (valu_pass: GRBM_GUI_ACTIVE, SQ_ACTIVE_INST_VALU, "
                                                         "SQ_THREAD_CYCLES_VALU of the same dispatches)"}
        r["binding"] = {
            "resource": "VALU issue (FP64 slab/Moeller-Trumbore arithmetic at ~half lane utilisation), with the "
                        "vector-memory data path (TA/TD) next: per-lane BVH record and triangle loads served from L1/L2",
            "valu_busy": prof.get("valu_busy"), "valu_lane_util": prof.get("valu_lane_util"),
            "td_busy": prof.get("td_busy"), "ta_busy": prof.get("ta_busy"),
            "note": "valu_busy = SQ_ACTIVE_INST_VALU/256 CUs / (GRBM_GUI_ACTIVE/8) (rocprofiler-sdk VALUBusy); "
                    "td_busy = TD_TD_BUSY_sum/256 / (GRBM_GUI_ACTIVE/8); both from the same profile",
            "executed_load_bytes": int(load_bytes),
            "executed_load_GBs": round(load_bytes / (kernel_ms * 1e-3) / 1e9, 1)}
    # the pipelined loop's own per-frame GPU time: rocprofv3 --kernel-trace of this bench's timed
    # frames (16 in flight), union of the render launches' intervals per frame
    # (tools/overlap_session.sh + tools/overlap_summary.py -> profiles/overlap_<config>.json)
    opath = os.path.join(ROOT, "profiles", f"overlap_{args.config}.json")
    if os.path.exists(opath) and world == 1:
        with open(opath) as fh:
            ov = json.load(fh)
        pl = {"union_per_frame_ms": ov["union_per_frame_ms"], "concurrency": ov["concurrency"],
              "max_overlap": ov["max_overlap"], "idle_fraction_of_span": ov["idle_fraction_of_span"],
              "trace_bench_ms_per_step": ov.get("bench_ms_per_step"),
              "source": os.path.relpath(opath, ROOT),
              "profile_build_matches": ov.get("lib_sha256_16") == lib_sha,
              "what": "render launches of the timed frames under rocprofv3 --kernel-trace: union of their "
                      "[start, end) per frame (the GPU time a pipelined frame costs), mean launches running "
                      "at once, most at once; achieved = HBM bytes per launch / union per frame"}
        if r["traffic"] is not None:
            pl["achieved"] = round(r["traffic"] / (ov["union_per_frame_ms"] * 1e-3) / 1e9, 2)
            pl["frac"] = round(pl["achieved"] / HBM_PEAK_GBS, 4)
        if not pl["profile_build_matches"]:
            pl.pop("achieved", None)
            pl.pop("frac", None)
        r["pipelined"] = pl
    r["reference_work"] = {
        "what": "SURVEY.md 8(d) algorithmic bytes of the reference's unpruned walk (56 N_node + 72 N_tri + "
                "72 N_smooth + 24 N_px), counted on the GPU in reference order; most are cache hits, so the "
                "equivalent rate exceeds HBM peak and is NOT an HBM fraction",
        "bytes_per_launch": int(alg_bytes), "bytes_per_ray": round(alg_bytes / max(1, rays_rank), 1),
        "equiv_GBs": round(alg_bytes / (kernel_ms * 1e-3) / 1e9, 1),
        "counts": {"node_fetches": int(wc.ref_node_fetches), "tri_tests": int(wc.ref_tri_tests),
                   "smooth_hits": int(wc.ref_smooth_hits), "pixels": int(wc.ref_pixels)}}
    r["executed"] = {"records": int(wc.records_fetched), "tri_tests": int(wc.tri_tests),
                     "normal_fetches": int(wc.normal_fetches), "pixels": int(wc.pixels)}
    r["per_lane_record_loads"] = {
        "lane_loads": int(wc.divergent_lane_loads), "distinct_records": int(wc.divergent_distinct_records),
        "distinct_fraction": round(wc.divergent_distinct_records / max(1, wc.divergent_lane_loads), 4),
        "what": "inner steps with the wave's lanes at more than one record (vector loads): lane loads vs "
                "distinct records among the wave's lanes at that step"}
    r["simd_efficiency"] = {"closest": round(wc.lane_steps_closest / max(1, 64 * wc.wave_steps_closest), 3),
                            "shadow": round(wc.lane_steps_shadow / max(1, 64 * wc.wave_steps_shadow), 3)}
    r["iterations"] = {
        k: {"wave_iters_inner": int(wc.iter_wave_inner[q]), "wave_iters_leaf": int(wc.iter_wave_leaf[q]),
            "wave_iters_scalar": int(wc.iter_wave_scalar[q]), "lane_inner": int(wc.iter_lane_inner[q]),
            "lane_leaf": int(wc.iter_lane_leaf[q])}
        for q, k in enumerate(("closest", "shadow"))}
    r["iterations"]["what"] = ("walk iterations of the unified walks: wave iterations in which some lane took an inner "
                               "step / a leaf run / the wave-uniform scalar inner step, and lane iterations of each kind")
    r["lib_sha256_16"] = lib_sha
    return r


def _lib_sha():
    from myraytracer_amd.engine import LIB_PATH
    path = os.environ.get("MYRT_LIB") or LIB_PATH
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def side_paths(eng, first, step, rows, W, H, rays_rank, args):
    """FP64 [Vec3] frame (Renderer.render's output) delivered to page-locked host memory, and
    the launch alone with the image left in HBM (no delivery)."""
    import numpy as np
    import torch
    import myraytracer_amd as M
    res = {}
    rgb = M.pinned_array((H, W, 3), np.float64)
    eng.render_into(0, first, step, rgb=rgb, rgba=None, frame_layout=True)
    nh = 10
    t = time.perf_counter()
    for _ in range(nh):
        eng.render_into(0, first, step, rgb=rgb, rgba=None, frame_layout=True)
    ms = (time.perf_counter() - t) * 1e3 / nh
    res["fp64_path"] = {"ms_per_frame": round(ms, 4), "value": round(rays_rank / (ms * 1e-3) / 1e6, 2),
                        "what": "rt_render of the FP64 RGB framebuffer (24 B/px) into page-locked host memory"}
    del rgb
    out = torch.empty((max(rows, 1), W, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    for _ in range(3):
        eng.render_device(0, 0, first, step, stream=stream.cuda_stream, out_rgba_ptr=out.data_ptr())
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        eng.render_device(0, 0, first, step, stream=stream.cuda_stream, out_rgba_ptr=out.data_ptr())
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / 20
    res["device_only"] = {"ms_per_frame": round(ms, 4), "value": round(rays_rank / (ms * 1e-3) / 1e6, 2),
                          "what": "rt_render_device back to back, RGBA8 left in HBM (no delivery)"}
    return res


def cgroup_cpu_quota(path="/sys/fs/cgroup/cpu.max"):
    """CPUs the process may actually use: the cgroup v2 CPU quota (cpu.max = "quota period",
    or "max") - on the GPU box 1600000/100000 = 16 CPUs while the affinity mask shows all 256
    cores of the machine (profiles/r03a_cpu_probe.txt).  Returns (cpus or None, path, raw)."""
    try:
        with open(path) as fh:
            raw = fh.read().strip()
    except OSError:
        return None, path, None
    q, _, per = raw.partition(" ")
    if q == "max" or not per:
        return None, path, raw
    import math
    return max(1, math.ceil(int(q) / int(per))), path, raw


def cpu_threads(args):
    """Threads for the CPU baseline: the cores this process can really run on = min(affinity,
    cgroup quota).  Returns (threads, evidence)."""
    aff = len(os.sched_getaffinity(0))
    quota, qpath, raw = cgroup_cpu_quota()
    usable = min(aff, quota) if quota else aff
    ev = {"affinity": aff, "cgroup_cpu_max": raw, "cgroup_source": qpath, "cgroup_quota_cpus": quota,
          "usable_cores": usable, "nproc": os.cpu_count(), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
    return (args.cpu_threads or usable), ev


def cpu_baseline(scene, H, args):
    """Oracle (C++ restatement of the reference CPU renderer): median over whole frames at the
    CPU share (one task per 8-row chunk, Object+Extension.swift:285-360), plus 1 thread."""
    import oracle
    cores, evidence = cpu_threads(args)
    t0 = time.time()
    o = oracle.OracleScene(scene if scene.objects[0].ply_path is None else _inline(scene))
    build_s = time.time() - t0
    nchunks = (H + 7) // 8
    rates, px = [], 0
    for _ in range(max(1, args.cpu_frames)):
        _, st = o.render(0, 0, 1, threads=cores)
        rates.append((st.primary_rays + st.shadow_rays) / (st.milliseconds / 1e3) / 1e6)
        px = st.pixels
    stride = 16
    one = []
    for k in range(2):
        _, st = o.render(0, k, stride, threads=1)
        one.append((st.primary_rays + st.shadow_rays) / (st.milliseconds / 1e3) / 1e6)
    med = statistics.median(rates)
    return {"value": round(med, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
            "frames": [round(x, 3) for x in rates], "spread": round((max(rates) - min(rates)) / med, 3),
            "one_thread": round(statistics.median(one), 4),
            "cores_evidence": evidence,
            "sample": f"median of {len(rates)} whole frames ({px} px each) on {cores} threads = the cores this "
                      f"process may use (min of the affinity mask and the cgroup CPU quota, cores_evidence); "
                      f"one_thread = every "
                      f"{stride}th 8-row chunk on 1 thread, {len(one)} runs; rays = primary + shadow cast; "
                      f"oracle BVH build {build_s:.1f}s excluded"}


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
