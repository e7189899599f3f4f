"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): per-channel L-inf <= 1e-5 on the FP64 framebuffer,
plus exact RGBA8 equality.  Every test renders through libmyrt.so on cuda:0.
"""
import copy

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5   # per-channel L-inf, north_star


def _compare(sc, chunk_first=0, chunk_step=1, cam=0, tol=TOL, check_rgba=True, options=None):
    eng = M.RayTracerEngine(sc)
    for k, v in (options or {}).items():
        eng.set_option(k, v)
    rgb, rgba, st = eng.render_rows(cam, chunk_first, chunk_step, True)
    o = oracle.OracleScene(sc)
    ref, ref8, ost = o.render(cam, chunk_first, chunk_step, threads=0, rgba=True)
    diff = np.abs(rgb - ref)
    linf = float(diff.max()) if diff.size else 0.0
    bad = int((diff > tol).any(axis=-1).sum())
    assert linf <= tol, f"L-inf {linf:.3e} over {bad} pixels (of {diff.shape[0] * diff.shape[1]})"
    if check_rgba:
        assert np.array_equal(rgba, ref8), f"RGBA8 mismatch on {int((rgba != ref8).any(axis=-1).sum())} pixels"
    assert st.primary_rays == ost.primary_rays
    assert st.shadow_rays == ost.shadow_rays, (st.shadow_rays, ost.shadow_rays)
    assert st.secondary_rays == ost.secondary_rays, (st.secondary_rays, ost.secondary_rays)
    # shadow walks actually run: the kernels skip the ones whose result the reference discards (N.L <= 0)
    assert st.shadow_rays_traced == ost.shadow_rays_used, (st.shadow_rays_traced, ost.shadow_rays_used)
    eng.close()
    return linf, st


def test_c1_single_triangle_full():
    linf, st = _compare(scenes.scene_c1())
    assert st.primary_rays == 256 * 256


def test_c2_bunny_standin_reduced():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 320, 240)
    _compare(sc)


def test_c2_from_ply(scene_dir):
    # product loads the PLY itself; oracle gets the same float32-widened arrays inline
    sc_ply = scenes.scaled(scenes.scene_c2(path_dir=scene_dir), 200, 150)
    sc_inl = scenes.scaled(scenes.scene_c2(inline=True), 200, 150)
    eng = M.RayTracerEngine(sc_ply)
    rgb, rgba, st = eng.render_rows(0, 0, 1, True)
    ref, ref8, _ = oracle.OracleScene(sc_inl).render(0, threads=0, rgba=True)
    assert float(np.abs(rgb - ref).max()) <= TOL
    assert np.array_equal(rgba, ref8)


def test_c2_full_resolution_sampled_rows():
    sc = scenes.scene_c2(inline=True)            # 800x600
    _compare(sc, chunk_first=3, chunk_step=7)


def test_c3_sampled_chunks():
    sc = scenes.scene_c3(inline=True)            # 1920x1080, ~1.02M tris
    _compare(sc, chunk_first=5, chunk_step=17)


def test_mirror_and_conductor_bounces():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 160, 120)
    sc.materials = [M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.3, 0.3, 0.3), specular=(0.5, 0.5, 0.5),
                               phong=16.0, mirror=(0.7, 0.6, 0.5), type="mirror"),
                    M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.3, 0.3, 0.3), specular=(0.5, 0.5, 0.5),
                               phong=16.0, mirror=(0.9, 0.8, 0.7), ior=1.5, absorption_index=2.5,
                               type="conductor")]
    ground = M.Mesh(id=7, material="2", positions=np.array([[-5, -1.3, -5], [5, -1.3, -5], [5, -1.3, 5],
                                                            [-5, -1.3, 5]], np.float64),
                    indices=np.array([[1, 3, 2], [1, 4, 3]], np.int32))
    sc.objects = sc.objects + [ground]
    sc.max_recursion_depth = 4
    _compare(sc)


def test_glossy_roughness_and_dof_multisample():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 96, 72)
    sc.materials = [M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.5, 0.4, 0.3), specular=(0.5, 0.5, 0.5),
                               phong=8.0, mirror=(0.5, 0.5, 0.5), roughness=0.15, type="mirror")]
    c = sc.cameras[0]
    c.num_samples = 4
    c.aperture_size = 0.05
    c.focus_distance = 4.0
    _compare(sc)


def test_non_square_spp_quirk():
    # numSamples = 5 -> n = 2: 4 samples taken, divided by 5 (Object+Extension.swift:300-354)
    sc = scenes.scene_c1(48, 40)
    sc.cameras[0].num_samples = 5
    _compare(sc)


def test_multi_mesh_instances_and_translation():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 120, 90)
    base = sc.objects[0]
    sc.objects = [base,
                  M.MeshInstance(id=11, base_mesh_id=base.id, material="1", transform=M.translation(1.5, 0.0, -1.0)),
                  M.MeshInstance(id=12, base_mesh_id=11, material=None, transform=M.translation(-1.5, 0.25, -2.0)),
                  M.Triangle(vertices=((-3, -1, -3), (3, -1, -3), (0, 2, -3.5)), material="1")]
    _compare(sc)


def test_motion_blur_instance():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 80, 60)
    base = sc.objects[0]
    sc.objects = [base, M.MeshInstance(id=21, base_mesh_id=base.id, material="1",
                                       transform=M.translation(0.5, 0.0, 0.5), motion_blur=(0.3, 0.0, 0.0))]
    base.motion_blur = (0.0, 0.1, 0.0)
    _compare(sc)


def test_nearplane_camera_and_no_fovy():
    sc = scenes.scene_c1(64, 48)
    c = sc.cameras[0]
    c.type = "simple"
    c.gaze = (0.0, 0.0, -1.0)
    c.near_plane = (-0.6, 0.6, -0.45, 0.45)
    _compare(sc)
    sc2 = scenes.scene_c1(64, 48)
    sc2.cameras[0].fovy = None
    _compare(sc2)


def test_empty_scene_is_black_and_miss_background():
    sc = scenes.scene_c1(32, 16)
    sc.objects = []
    eng = M.RayTracerEngine(sc)
    r = eng.render(0)
    assert np.all(r.rgb == 0.0)          # no TLAS -> trace returns .zero (Object+Extension.swift:98)
    ref, _ = oracle.OracleScene(sc).render(0)
    assert np.array_equal(r.rgb, ref)


def test_invalid_camera_error():
    eng = M.RayTracerEngine(scenes.scene_c1(16, 16))
    with pytest.raises(M.RenderError) as e:
        eng.render(3)
    assert e.value.code == -10


def test_two_replicas_gather_matches_single():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 128, 100)   # 13 chunks, last partial
    one = M.RayTracerEngine(sc, devices=[0]).render(0)
    two = M.RayTracerEngine(sc, devices=[0, 0]).render(0)       # two replicas, round-robin chunks
    assert np.array_equal(one.rgb, two.rgb)
    assert np.array_equal(one.rgba8, two.rgba8)
    assert one.stats.shadow_rays == two.stats.shadow_rays


@pytest.mark.parametrize("devices,first,step", [([0], 0, 1), ([0], 1, 3), ([0, 0], 0, 1), ([0, 0, 0], 2, 2)])
def test_pinned_outputs_take_direct_dma(devices, first, step):
    """rt_render into page-locked caller buffers (rt_host_alloc): rows are DMA'd straight into
    them, coalesced per run of adjacent chunks; results equal the pageable (staged) path."""
    sc = scenes.scaled(scenes.scene_c2(inline=True), 136, 100)  # 13 chunks, last partial
    eng = M.RayTracerEngine(sc, devices=devices)
    rgb_p, rgba_p, st_p = eng.render_rows(0, first, step, True)
    prgb, prgba = eng.alloc_frame(0, first, step)
    prgb.fill(-1.0)
    prgba.fill(7)
    rgb_d, rgba_d, st_d = eng.render_rows(0, first, step, True, out=prgb, out_rgba=prgba)
    assert rgb_d is prgb and rgba_d is prgba
    assert np.array_equal(rgb_d, rgb_p) and np.array_equal(rgba_d, rgba_p)
    assert (st_d.primary_rays, st_d.shadow_rays) == (st_p.primary_rays, st_p.shadow_rays)
    # RGB only, then progress reaches the total
    seen = []
    prgb.fill(-1.0)
    eng.render_rows(0, first, step, False, progress=lambda p: seen.append(p.fraction) or True, out=prgb)
    assert np.array_equal(prgb, rgb_p) and seen and seen[-1] == 1.0
    eng.close()


def test_device_path_matches_host_path():
    import torch
    sc = scenes.scaled(scenes.scene_c2(inline=True), 200, 120)
    eng = M.RayTracerEngine(sc)
    host = eng.render(0).rgb
    out = torch.empty((120, 200, 3), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()
    eng.render_device(out.data_ptr(), 0, 0, 1, stream=stream.cuda_stream)
    stream.synchronize()
    assert np.array_equal(out.cpu().numpy(), host)
    wc = eng.work_counters(out.data_ptr(), 0, 0, 1, stream=stream.cuda_stream)
    assert wc.pixels == 200 * 120 and wc.records_fetched > 0 and wc.tri_tests > 0


def _ref_counts_case(name):
    if name == "c2":
        return scenes.scaled(scenes.scene_c2(inline=True), 160, 120), 0, 1
    if name == "c3":
        return scenes.scene_c3(inline=True), 2, 23
    if name == "instances":
        sc = scenes.scaled(scenes.scene_c2(inline=True), 96, 64)
        base = sc.objects[0]
        sc.objects = [base,
                      M.MeshInstance(id=11, base_mesh_id=base.id, material="1", transform=M.translation(1.5, 0.0, -1.0)),
                      M.Triangle(vertices=((-3, -1, -3), (3, -1, -3), (0, 2, -3.5)), material="1")]
        return sc, 0, 1
    sc = scenes.scaled(scenes.scene_c2(inline=True), 96, 64)      # mirror bounces
    sc.materials[0].type = "mirror"
    sc.materials[0].mirror = (0.5, 0.5, 0.5)
    sc.max_recursion_depth = 3
    return sc, 0, 1


@pytest.mark.parametrize("case", ["c2", "c3", "instances", "mirror"])
def test_reference_order_work_counts_match_oracle(case):
    """The GPU's reference-order tally (the roofline's algorithmic bytes)
    equals the oracle's instrumented counts exactly."""
    import torch
    sc, first, step = _ref_counts_case(case)
    eng = M.RayTracerEngine(sc)
    W, H = sc.cameras[0].image_resolution
    rows = M.rows_for_chunks(H, first, step)
    out = torch.empty((rows, W, 3), dtype=torch.float64, device="cuda")
    wc = eng.work_counters(out.data_ptr(), 0, first, step)
    _, ost = oracle.OracleScene(sc).render(0, first, step, threads=0)
    got = (wc.ref_node_fetches, wc.ref_tri_tests, wc.ref_smooth_hits, wc.ref_pixels)
    want = (ost.node_fetches, ost.tri_tests, ost.smooth_hits, ost.pixels)
    assert got == want
    assert wc.records_fetched > 0 and wc.pixels == wc.ref_pixels
