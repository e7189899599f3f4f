"""Full-frame GPU parity on exactly what bench.py times, and the multi-GPU gather.

* C3 (1.02M tris, 1920x1080) loaded from its PLY with default settings, rendered through
  rt_render_ex into page-locked whole-frame buffers (the bench's headline path: the kernels
  store the rows into host memory) and through rt_render_device (the device-only side path),
  each compared on the FULL frame with the oracle ("check all of C1-C3").
* C2 at its full 800x600.
* C4: the C3 frame rendered by 8 replicas (chunk c on replica c mod 8), equal to the oracle and
  to the 1-replica frame; disjoint chunk selections gathered into one frame (frame layout).
* bench.py --gpus 2 (two ranks on this one GPU): the strong split gathers a complete frame
  bit-identical to the 1-GPU frame.
Bar: per-channel L-inf <= 1e-5 on FP64, exact RGBA8, equal ray counts.
"""
import copy
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _inline(scene):
    """The PLY-loaded scene as inline arrays read by the product's PLY reader (the oracle takes
    arrays; the reader itself is pinned against the reference's CPly, tests/test_ply.py)."""
    s = copy.deepcopy(scene)
    for obj in s.objects:
        if isinstance(obj, M.Mesh) and obj.ply_path is not None:
            m = M.ply_load(obj.ply_path)
            obj.positions, obj.indices, obj.normals = m["positions"], m["indices"], m["normals"]
            obj.indices_one_based = False
            obj.ply_path = None
    return s


@pytest.fixture(scope="module")
def c3_ply(scene_dir):
    sc = scenes.scene_c3(path_dir=scene_dir)
    ref, ref8, ost = oracle.OracleScene(_inline(sc)).render(0, threads=0, rgba=True)
    return sc, ref, ref8, ost


def _assert_frame(rgb, rgba, ref, ref8):
    if rgb is not None:
        d = np.abs(rgb - ref)
        assert float(d.max()) <= TOL, f"L-inf {float(d.max()):.3e} on {int((d > TOL).any(-1).sum())} px"
    if rgba is not None:
        assert np.array_equal(rgba, ref8), f"RGBA8 differs on {int((rgba != ref8).any(-1).sum())} px"


@pytest.mark.parametrize("wide", [1, 0])
def test_c3_full_frame_bench_path(c3_ply, wide):
    """The bench's own call on the full C3 frame, through the four-wide walk (default) and the
    binary walk (render option wide = 0)."""
    sc, ref, ref8, ost = c3_ply
    eng = M.RayTracerEngine(sc)
    eng.set_option("wide", wide)
    H, W = ref.shape[:2]
    rgba = M.pinned_array((H, W, 4), np.uint8)
    rgb = M.pinned_array((H, W, 3), np.float64)
    rgba.fill(0)
    st = eng.render_into(0, 0, 1, rgb=None, rgba=rgba, frame_layout=True)     # bench.py's headline call
    _assert_frame(None, rgba, ref, ref8)
    assert st.primary_rays == ost.primary_rays and st.shadow_rays == ost.shadow_rays
    assert st.shadow_rays_traced == ost.shadow_rays_used
    st2 = eng.render_into(0, 0, 1, rgb=rgb, rgba=None, frame_layout=True)     # fp64 side path
    _assert_frame(rgb, None, ref, ref8)
    assert st2.shadow_rays_traced == st.shadow_rays_traced
    eng.close()


def test_c3_full_frames_in_flight_bench_path(c3_ply):
    """bench.py's timed loop exactly: frames submitted with 4 renders in flight
    (engine.frame_pipeline -> rt_render_submit / rt_render_wait), frame k into page-locked
    framebuffer k mod 4; every delivered frame equals the oracle's RGBA8 and its counts."""
    import collections
    sc, ref, ref8, ost = c3_ply
    eng = M.RayTracerEngine(sc)
    H, W = ref.shape[:2]
    fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(4)]
    submit, wait = eng.frame_pipeline(0, 0, 1, fbs, frame_layout=True)
    pend = collections.deque()
    done = 0

    def check(k, st):
        _assert_frame(None, fbs[k % 4], ref, ref8)
        assert st.shadow_rays == ost.shadow_rays and st.shadow_rays_traced == ost.shadow_rays_used
        fbs[k % 4].fill(0)

    for k in range(10):
        if len(pend) == 4:
            kk, t = pend.popleft()
            check(kk, wait(t))
            done += 1
        fbs[k % 4].fill(0) if k < 4 else None
        pend.append((k, submit(k)))
    while pend:
        kk, t = pend.popleft()
        check(kk, wait(t))
        done += 1
    assert done == 10
    eng.close()


def test_c3_full_frame_device_path(c3_ply):
    import torch
    sc, ref, ref8, _ = c3_ply
    eng = M.RayTracerEngine(sc)
    H, W = ref.shape[:2]
    out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    out8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    eng.render_device(out.data_ptr(), 0, 0, 1, stream=s.cuda_stream, out_rgba_ptr=out8.data_ptr())
    s.synchronize()
    _assert_frame(out.cpu().numpy(), out8.cpu().numpy(), ref, ref8)
    eng.close()


def test_c4_eight_replicas_full_c3(c3_ply):
    """configs[3]: the C3 frame split over 8 replicas (8-row chunk c on replica c mod 8; here all
    on the one GPU of the box), gathered by rt_render into one page-locked frame."""
    sc, ref, ref8, ost = c3_ply
    H, W = ref.shape[:2]
    eng8 = M.RayTracerEngine(sc, devices=[0] * 8)
    rgb = M.pinned_array((H, W, 3), np.float64)
    rgba = M.pinned_array((H, W, 4), np.uint8)
    rgb.fill(-1.0)
    rgba.fill(0)
    st = eng8.render_into(0, 0, 1, rgb=rgb, rgba=rgba)
    _assert_frame(rgb, rgba, ref, ref8)
    assert st.shadow_rays == ost.shadow_rays and st.shadow_rays_traced == ost.shadow_rays_used
    # the staged path (pageable buffers) gathers the same image
    r2, r28, _ = eng8.render_rows(0, 0, 1, True)
    assert np.array_equal(r2, rgb) and np.array_equal(r28, rgba)
    eng8.close()


def test_c2_full_frame():
    sc = scenes.scene_c2(inline=True)            # 800x600, every chunk
    eng = M.RayTracerEngine(sc)
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    _assert_frame(rgb, rgba, ref, ref8)
    assert (st.primary_rays, st.shadow_rays) == (ost.primary_rays, ost.shadow_rays)
    eng.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_frame_layout_gathers_disjoint_selections(devices):
    """RT_RENDER_FRAME_LAYOUT: selections k, k+3, ... (k = 0, 1, 2) fill one whole frame; rows
    outside a selection are left untouched."""
    sc = scenes.scaled(scenes.scene_c2(inline=True), 136, 100)     # 13 chunks, last partial
    eng = M.RayTracerEngine(sc, devices=devices)
    full, full8, _ = eng.render_rows(0, 0, 1, True)
    for pinned in (True, False):
        if pinned:
            rgb, rgba = M.pinned_array((100, 136, 3), np.float64), M.pinned_array((100, 136, 4), np.uint8)
        else:
            rgb, rgba = np.empty((100, 136, 3)), np.empty((100, 136, 4), np.uint8)
        rgb.fill(-7.0)
        rgba.fill(3)
        eng.render_into(0, 1, 3, rgb=rgb, rgba=rgba, frame_layout=True)
        sel = np.zeros(100, bool)
        for c in range(1, 13, 3):
            sel[8 * c: 8 * c + 8] = True
        assert np.array_equal(rgb[sel], full[sel]) and np.array_equal(rgba[sel], full8[sel])
        assert np.all(rgb[~sel] == -7.0) and np.all(rgba[~sel] == 3)
        for k in (0, 2):
            eng.render_into(0, k, 3, rgb=rgb, rgba=rgba, frame_layout=True)
        assert np.array_equal(rgb, full) and np.array_equal(rgba, full8)
    eng.close()


def _bench(args, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_strong_split_two_ranks_gathers_the_same_frame():
    """`bench.py --gpus 2` (torchrun started by bench.py, both ranks pinned to this GPU): one C2
    frame per step, chunks split over the ranks, rows stored into one shared page-locked
    framebuffer - complete and bit-identical to the 1-GPU frame."""
    common = ["--config", "c2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-side-paths"]
    one = _bench(["--gpus", "1"] + common, {})
    two = _bench(["--gpus", "2"] + common, {"MYRT_BENCH_DEVICE": "0"})
    two_staged = _bench(["--gpus", "2", "--gather", "staged"] + common, {"MYRT_BENCH_DEVICE": "0"})
    assert two_staged["gather"]["rgba8_sha256"] == one["gather"]["rgba8_sha256"]
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert one["gather"]["rows_complete"] and two["gather"]["rows_complete"]
    assert two["gather"]["rgba8_sha256"] == one["gather"]["rgba8_sha256"]
    assert two["rays"]["per_step"] == one["rays"]["per_step"]


@pytest.mark.timeout(600)
def test_bench_strong_split_eight_ranks_on_one_gpu():
    """The C4 process path at N = 8 (Object+Extension.swift:75-82): `bench.py --gpus 8` with
    every rank pinned to this GPU (MYRT_BENCH_DEVICE=0, 32 / 8 = 4 hardware queues per rank),
    C2, 3 steps: 8 processes, 16 shared registered framebuffers, chunk c on rank c mod 8.  The
    gathered frame is complete and bit-identical to the 1-GPU frame, and the line carries
    every rank's timing."""
    common = ["--config", "c2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-side-paths"]
    one = _bench(["--gpus", "1"] + common, {})
    eight = _bench(["--gpus", "8"] + common, {"MYRT_BENCH_DEVICE": "0"})
    assert eight["n_gpus"] == 8 and eight["scaling"] == "strong"
    assert eight["config"]["hw_queues"] == "4"
    assert eight["gather"]["rows_complete"]
    assert eight["gather"]["rgba8_sha256"] == one["gather"]["rgba8_sha256"]
    assert eight["rays"]["per_step"] == one["rays"]["per_step"]
    pr = eight["per_rank"]
    assert len(pr["ms_per_step"]) == 8 and pr["max_ms"] >= pr["min_ms"] > 0
    assert len(pr["device_ms_per_frame"]) == 8 and min(pr["device_ms_per_frame"]) > 0
    assert sum(pr["rows"]) == 600 and all(x > 0 for x in pr["submit_us_per_frame"])
    # staged gather: each GPU's DMA engine delivers into a private frame, the rank's host thread
    # copies its rows into the shared frame - the same image
    staged = _bench(["--gpus", "8", "--gather", "staged"] + common, {"MYRT_BENCH_DEVICE": "0"})
    assert staged["gather"]["mode"] == "staged" and staged["gather"]["rows_complete"]
    assert staged["gather"]["rgba8_sha256"] == one["gather"]["rgba8_sha256"]
    assert staged["per_rank"]["gather"] == "staged" and len(staged["per_rank"]["device_ms_per_frame"]) == 8
    # NUMA: every rank's GPU node, CPU affinity and the node of its frame pages;
    # the opt-in first-touch placement (each rank binds to its GPU's node and touches its own rows
    # before registration) gathers the same image
    for line in (eight, staged):
        assert len(line["per_rank"]["numa"]) == 8
        for r in line["per_rank"]["numa"]:
            assert "node" in r["gpu"] and r["affinity"] and "frame_pages_by_node" in r
    assert sum(sum(r["frame_pages_by_node"].values()) for r in eight["per_rank"]["numa"]) > 0
    placed = _bench(["--gpus", "8", "--numa-placement", "first-touch"] + common, {"MYRT_BENCH_DEVICE": "0"})
    assert placed["gather"]["rows_complete"]
    assert placed["gather"]["rgba8_sha256"] == one["gather"]["rgba8_sha256"]
    assert all(r["placement"] == "first-touch" for r in placed["per_rank"]["numa"])
    assert one["numa"]["gpu"] is not None and "scratch_bytes_after_warmup" in one["scene"]


@pytest.mark.timeout(400)
@pytest.mark.parametrize("name", ["c3i", "c3i_tw", "c3g", "c3d", "c3r"])
def test_general_path_bench_configs_full_frame(scene_dir, name):
    """The bench's general-path configs on full 1920x1080 frames against the oracle: C3i (C3's
    geometry as 25 transformed mesh instances: the literal TLAS->BLAS walk, RTContext.swift:
    619-720; the flattened instance tree, and tw_walk with option fit = 0) and C3g (glass spheres + two area lights: render_full with k_events/k_jscan,
    Object+Extension.swift:145-251) and C3d (the glass spheres with the point light only: level
    passes + node shading without events), through bench.py's call (RGBA8 into page-locked
    memory) and the FP64 frame."""
    make = {"c3i": scenes.scene_c3_instanced, "c3i_tw": scenes.scene_c3_instanced, "c3g": scenes.scene_c3_glass,
            "c3r": lambda path_dir: scenes.scene_c3_glass(path_dir=path_dir, rough=True),
            "c3d": lambda path_dir: scenes.scene_c3_glass(path_dir=path_dir, area_lights=False)}[name]
    sc = make(path_dir=scene_dir)
    ref, ref8, ost = oracle.OracleScene(_inline(sc)).render(0, threads=0, rgba=True)
    eng = M.RayTracerEngine(sc)
    if name == "c3i_tw":
        eng.set_option("fit", 0)
    H, W = ref.shape[:2]
    rgba = M.pinned_array((H, W, 4), np.uint8)
    rgba.fill(0)
    st = eng.render_into(0, 0, 1, rgb=None, rgba=rgba, frame_layout=True)
    _assert_frame(None, rgba, ref, ref8)
    assert (st.primary_rays, st.shadow_rays, st.secondary_rays) == \
        (ost.primary_rays, ost.shadow_rays, ost.secondary_rays)
    rgb, _, _ = eng.render_rows(0, 0, 1, False)
    _assert_frame(rgb, None, ref, ref8)
    eng.close()
