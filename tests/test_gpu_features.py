"""GPU parity for the trace() branches beyond the fast megakernel:
spheres and planes (RTContext.swift:122-192, 513-538, 851-870), dielectric materials with
two child rays per bounce and Beer absorption (Object+Extension.swift:207-251), and area
lights with the chunk-sequential jitterIndex (:145-186, :288).  Same bar as
test_gpu_parity.py: per-channel L-inf <= 1e-5, exact RGBA8, equal ray counts."""
import copy

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import _abi as A
from myraytracer_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _compare(sc, chunk_first=0, chunk_step=1, cam=0, options=None):
    eng = M.RayTracerEngine(sc)
    for k, v in (options or {}).items():                 # render options (rt_scene_set_option)
        eng.set_option(k, v)
    rgb, rgba, st = eng.render_rows(cam, chunk_first, chunk_step, True)
    ref, ref8, ost = oracle.OracleScene(sc).render(cam, chunk_first, chunk_step, threads=0, rgba=True)
    diff = np.abs(rgb - ref)
    linf = float(diff.max()) if diff.size else 0.0
    assert linf <= TOL, f"L-inf {linf:.3e} on {int((diff > TOL).any(axis=-1).sum())} pixels"
    assert np.array_equal(rgba, ref8), f"RGBA8 mismatch on {int((rgba != ref8).any(axis=-1).sum())} pixels"
    assert (st.primary_rays, st.shadow_rays, st.secondary_rays) == \
        (ost.primary_rays, ost.shadow_rays, ost.secondary_rays)
    eng.close()
    return st


def scale_translate(s, tx, ty, tz):
    return (s, 0, 0, 0, 0, s, 0, 0, 0, 0, s, 0, tx, ty, tz, 1)


def _materials():
    return [M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.6, 0.5, 0.4), specular=(0.4, 0.4, 0.4), phong=24.0),
            M.Material(ambient=(0.05, 0.05, 0.05), diffuse=(0.2, 0.2, 0.2), specular=(0.6, 0.6, 0.6), phong=64.0,
                       mirror=(0.7, 0.7, 0.75), type="mirror"),
            M.Material(ambient=(0.0, 0.0, 0.0), diffuse=(0.1, 0.1, 0.1), specular=(0.5, 0.5, 0.5), phong=50.0,
                       ior=1.5, absorption=(0.05, 0.1, 0.2), type="dielectric"),
            M.Material(ambient=(0.05, 0.05, 0.05), diffuse=(0.2, 0.2, 0.2), specular=(0.5, 0.5, 0.5), phong=30.0,
                       mirror=(0.9, 0.8, 0.6), ior=0.2, absorption_index=3.0, type="conductor"),
            M.Material(ambient=(0.0, 0.0, 0.0), diffuse=(0.1, 0.1, 0.1), specular=(0.3, 0.3, 0.3), phong=20.0,
                       ior=1.33, roughness=0.08, type="dielectric")]


def _primitives_scene(w=160, h=120):
    cam = M.Camera(position=(0.0, 1.0, 6.0), gaze_point=(0.0, 0.3, 0.0), up=(0.0, 1.0, 0.0), fovy=50.0,
                   image_resolution=(w, h))
    objs = [M.Plane(center=(0.0, -1.0, 0.0), normal=(0.0, 1.0, 0.0), material="1"),
            M.Sphere(center=(-1.6, 0.0, 0.0), radius=1.0, material="2"),
            M.Sphere(center=(0.0, 0.0, 0.0), radius=0.5, material="4", transform=scale_translate(2.0, 0.4, 0.0, -1.5)),
            M.Sphere(center=(1.7, -0.2, 0.8), radius=0.8, material="1"),
            M.Triangle(vertices=((-3.0, -1.0, -3.0), (3.0, -1.0, -3.0), (0.0, 2.5, -3.2)), material="1")]
    return M.Scene(cameras=[cam], materials=_materials(), objects=objs,
                   point_lights=[M.PointLight((4.0, 6.0, 5.0), (4000.0, 4000.0, 4000.0)),
                                 M.PointLight((-5.0, 3.0, 2.0), (1500.0, 1200.0, 1000.0))],
                   ambient_light=(20.0, 20.0, 20.0), background_color=(5.0, 10.0, 20.0),
                   shadow_ray_epsilon=1e-3, intersection_test_epsilon=1e-6, max_recursion_depth=4)


def test_spheres_planes_mirror_conductor():
    _compare(_primitives_scene())


def test_dielectric_spheres_and_mesh():
    sc = _primitives_scene(128, 96)
    sc.objects[1].material = "3"                       # glass sphere with absorption
    sc.objects[3].material = "5"                       # rough water-like sphere
    bunny = scenes.scaled(scenes.scene_c2(inline=True), 8, 8).objects[0]
    bunny.material = "3"
    bunny.transform = scale_translate(0.5, 1.8, 0.0, 1.5)
    sc.objects.append(bunny)
    sc.max_recursion_depth = 5
    st = _compare(sc)
    assert st.secondary_rays > 0


def test_dielectric_total_internal_reflection_depth_limit():
    sc = _primitives_scene(96, 72)
    for o in sc.objects[1:4]:
        o.material = "3"
    sc.max_recursion_depth = 2
    _compare(sc)


def _area_scene(w=120, h=90, spp=1):
    sc = _primitives_scene(w, h)
    sc.area_lights = [M.AreaLight(position=(0.0, 4.0, 1.0), normal=(0.0, -1.0, 0.0), radiance=(40.0, 38.0, 30.0),
                                  size=1.5),
                      M.AreaLight(position=(-3.0, 2.5, 3.0), normal=(0.5, -0.5, -0.5), radiance=(10.0, 12.0, 20.0),
                                  size=0.8)]
    sc.cameras[0].num_samples = spp
    return sc


def test_area_lights_jitter_index_full_frame():
    _compare(_area_scene())


def test_area_lights_sampled_chunks_multisample():
    # jitterIndex restarts per 8-row chunk, so any chunk selection must match the oracle
    _compare(_area_scene(104, 77, spp=4), chunk_first=1, chunk_step=3)


def test_area_lights_with_dielectric_and_mesh():
    sc = _area_scene(96, 64)
    sc.objects[1].material = "3"
    base = scenes.scaled(scenes.scene_c2(inline=True), 8, 8).objects[0]
    base.material = "1"
    base.transform = scale_translate(0.6, 0.0, 0.2, 1.8)
    sc.objects.append(base)
    _compare(sc)


@pytest.mark.parametrize("slots, nodeshade, lists", [(-1, 1, 1), (-1, 1, 0), (-1, 0, 1), (1, 1, 1), (8, 1, 1),
                                                     (0, 1, 1)])
def test_area_light_hit_log(slots, nodeshade, lists):
    """render_full reads the closest hits k_events logged instead of walking them again
    (RenderParams::hits), and k_shade shades the logged hits node-parallel (option nodeshade = 1,
    default) or render_full does (0): the default log holds every walk of the paths here, 8 or
    1 slots send longer paths past the log to the fallback walk, 0 turns the log off.  Glass, mirror and a rough
    dielectric give paths of up to 2^5 - 1 walks; four samples per pixel.  The rough material keeps
    the depth-first k_events: node shading runs over the list of logged hits it flags (option
    node_lists = 1, default) or per (tile, walk)."""
    # hitlog -1: sized to the scene's path trees (here 31 per sample); nodeshade: logged hits shaded
    # node-parallel (k_shade) or by render_full
    sc = _area_scene(88, 64, spp=4)
    sc.objects[1].material = "3"
    sc.objects[2].material = "2"
    sc.objects[3].material = "5"
    sc.max_recursion_depth = 4
    st = _compare(sc, options={"hitlog": slots, "nodeshade": nodeshade, "node_lists": lists})
    assert st.secondary_rays > 0


@pytest.mark.parametrize("levels, ppw, lists", [(1, 4, 1), (1, 4, 0), (1, 1, 0), (1, 64, 0), (0, 4, 1)])
@pytest.mark.parametrize("spp, depth, glass", [(1, 4, True), (4, 3, True), (1, 5, True), (4, 4, False), (9, 2, True)])
def test_area_light_level_passes(levels, ppw, lists, spp, depth, glass):
    """Breadth-first events passes (render_full.h k_level, option levels = 1, default) against the
    depth-first k_events (0): no rough material, so the tree's walks may run level by level;
    heap-indexed trees with glass (2^(D+1) - 1 nodes per traced sample), chains without; 4 and 9
    samples per pixel give several trees per pixel; depth 5 with one sample fills 63 of the 64
    log slots.  k_jofs must reproduce the depth-first jitterIndex offsets exactly.  Levels past 0
    and the node shading run over compacted node lists (option node_lists = 1, default: k_clist,
    k_level_c, k_shade_c; several traced samples give a level several spans of the log) or per
    tile, a wave running 1, 4 (default) or all of a level's node positions (option tree_ppw)."""
    sc = _area_scene(70, 56, spp=spp)                   # width 70: ragged last tile column
    sc.objects[1].material = "3" if glass else "2"
    sc.objects[2].material = "4"
    sc.objects[3].material = "3" if glass else "4"
    sc.max_recursion_depth = depth
    st = _compare(sc, options={"levels": levels, "tree_ppw": ppw, "node_lists": lists})
    assert st.secondary_rays > 0


@pytest.mark.parametrize("levels, lists", [(1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("spp, depth", [(1, 4), (4, 3)])
def test_dielectric_level_passes_without_area_lights(levels, lists, spp, depth):
    """Glass + mirror + conductor with point lights only: the level passes and node shading
    (option levels = 1, default; over compacted node lists or per tile, option node_lists) or
    render_full alone (levels = 0).  No jitterIndex here, so no events prefix."""
    sc = _primitives_scene(80, 60)
    sc.cameras[0].num_samples = spp
    sc.objects[1].material = "3"
    sc.objects[3].material = "3"
    sc.max_recursion_depth = depth
    st = _compare(sc, options={"levels": levels, "node_lists": lists})
    assert st.secondary_rays > 0


def test_c5_10m_mirrors_sampled_chunks_and_full_frame(scene_dir):
    """C5 (BASELINE configs[4]): ~10M triangles in two meshes (TLAS of 2), 3840x2160,
    depth-4 mirror reflections.  SURVEY.md §8d: 'for C5 check a sampled 1/64 of the rows
    plus the full image once'."""
    sc_ply = scenes.scene_c5(path_dir=scene_dir)
    eng = M.RayTracerEngine(sc_ply)
    orc = oracle.OracleScene(scenes.scene_c5(inline=True))
    for first, step in ((100, 64), (0, 1)):
        rgb, rgba, st = eng.render_rows(0, first, step, True)
        ref, ref8, ost = orc.render(0, first, step, threads=0, rgba=True)
        assert float(np.abs(rgb - ref).max()) <= TOL
        assert np.array_equal(rgba, ref8)
        assert (st.shadow_rays, st.secondary_rays) == (ost.shadow_rays, ost.secondary_rays)
        assert st.secondary_rays > 0
        del rgb, rgba, ref, ref8
    eng.close()


def test_progress_per_batch_and_cancel():
    """rt_render reports progress after every finished batch of chunks and honours
    cancellation (the reference's progress closure returns Bool, RayTracer.swift:115-131;
    SURVEY.md §8b: cancel at chunk granularity)."""
    sc = scenes.scaled(scenes.scene_c2(inline=True), 160, 200)      # 25 chunks -> 7 batches
    eng = M.RayTracerEngine(sc)
    seen = []
    r = eng.render(0, progress=lambda p: seen.append(p.fraction) or True)
    assert len(seen) >= 2 and seen == sorted(seen) and seen[-1] == 1.0
    ref = oracle.OracleScene(sc).render(0, threads=0)[0]
    assert float(np.abs(r.rgb - ref).max()) <= TOL
    calls = []
    with pytest.raises(M.RenderError) as e:
        eng.render(0, progress=lambda p: calls.append(p.fraction) or False)
    assert e.value.code == -60 and len(calls) == 1
    again = eng.render(0)                                            # the engine stays usable
    assert np.array_equal(again.rgb, r.rgb)


def test_second_camera_and_empty_selection():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 96, 64)
    c2 = copy.deepcopy(sc.cameras[0])
    c2.position = (1.5, 1.0, 3.5)
    c2.image_resolution = (72, 40)                                   # 5 chunks
    sc.cameras.append(c2)
    eng = M.RayTracerEngine(sc)
    rgb, rgba, st = eng.render_rows(1, 0, 1, True)
    ref, ref8, _ = oracle.OracleScene(sc).render(1, threads=0, rgba=True)
    assert rgb.shape == (40, 72, 3) and float(np.abs(rgb - ref).max()) <= TOL and np.array_equal(rgba, ref8)
    empty, _, st0 = eng.render_rows(1, 7, 1, True)                   # chunk 7 is past the image
    assert empty.shape == (0, 72, 3) and st0.primary_rays == 0


@pytest.mark.parametrize("fname", ["mixed.json", "mixed.xml"])
def test_scene_file_through_the_engine(tmp_path, fname):
    """RayTracerEngine.init(from: url) (RayTracer.swift:30-34) on a scene file with every object kind:
    the product resolves and parses the PLY itself; the oracle gets the same arrays inline."""
    import os
    import shutil
    from myraytracer_amd import sceneio
    from test_sceneio import GOLDEN, inline_plys
    shutil.copy(os.path.join(GOLDEN, fname), tmp_path)
    V, F = scenes.icosphere(1)
    scenes.write_ply(str(tmp_path / "ico.ply"), V * 0.7, F)
    path = str(tmp_path / fname)
    eng = M.RayTracerEngine.from_file(path)
    ref_scene = inline_plys(eng.scene)
    for cam in range(len(eng.scene.cameras)):
        rgb, rgba, st = eng.render_rows(cam, 0, 1, True)
        ref, ref8, ost = oracle.OracleScene(ref_scene).render(cam, threads=0, rgba=True)
        assert float(np.abs(rgb - ref).max()) <= TOL
        assert np.array_equal(rgba, ref8)
        assert (st.primary_rays, st.shadow_rays, st.secondary_rays) == \
            (ost.primary_rays, ost.shadow_rays, ost.secondary_rays)
    res = eng.save_png(str(tmp_path / "out.png"), 0)
    assert os.path.getsize(tmp_path / "out.png") > 0 and res.file_name == "mixed_lookat.png"
    eng.close()


# ---------------------------------------------------------------- maxRecursionDepth > 16
def _mirror_corridor(depth, w=64, h=48, glass=False):
    """A mirror/conductor box corridor (x = +-1, y = +-2) along -z, camera looking mostly
    sideways: most rays bounce until maxRecursionDepth stops them (trace() :97, :189-206).
    Levels beyond kMaxDepthGPU = 16 live in the device deep-frame buffer (render_full.h)."""
    wall = lambda x, m: M.Mesh(id=int(10 + 5 * (x + 1)), material=m,
                               positions=np.array([[x, -2, 2], [x, 2, 2], [x, 2, -60], [x, -2, -60]], np.float64),
                               indices=np.array([[1, 2, 3], [1, 3, 4]], np.int32), shading_mode="flat")
    floor = M.Mesh(id=30, material="2", positions=np.array([[-1, -2, 2], [1, -2, 2], [1, -2, -60], [-1, -2, -60]],
                                                           np.float64),
                   indices=np.array([[1, 3, 2], [1, 4, 3]], np.int32), shading_mode="flat")
    ceiling = M.Mesh(id=31, material="4", positions=np.array([[-1, 2, 2], [1, 2, 2], [1, 2, -60], [-1, 2, -60]],
                                                             np.float64),
                     indices=np.array([[1, 2, 3], [1, 3, 4]], np.int32), shading_mode="flat")
    objs = [wall(-1.0, "2"), wall(1.0, "4"), floor, ceiling]
    if glass:
        objs.append(M.Sphere(center=(0.2, -1.2, -6.0), radius=0.6, material="3"))
    cam = M.Camera(position=(0.0, 0.0, 0.0), gaze_point=(1.0, -0.05, -0.25), up=(0.0, 1.0, 0.0), fovy=40.0,
                   image_resolution=(w, h))
    return M.Scene(cameras=[cam], materials=_materials(), objects=objs,
                   point_lights=[M.PointLight((0.0, 1.5, -4.0), (800.0, 800.0, 800.0))],
                   ambient_light=(20.0, 20.0, 20.0), background_color=(5.0, 10.0, 20.0),
                   shadow_ray_epsilon=1e-3, intersection_test_epsilon=1e-6, max_recursion_depth=depth)


@pytest.mark.parametrize("depth", [17, 40])
def test_deep_mirror_recursion(depth):
    st = _compare(_mirror_corridor(depth))
    # most primary rays run to the depth limit: far more secondary rays than 16 per pixel allow
    assert st.secondary_rays > 16 * 64 * 48 // 2


def test_deep_recursion_with_glass_and_area_light():
    sc = _mirror_corridor(24, 48, 36, glass=True)
    sc.area_lights = [M.AreaLight(position=(0.0, 1.9, -5.0), normal=(0.0, -1.0, 0.0), size=0.8,
                                  radiance=(60.0, 60.0, 60.0))]
    _compare(sc)


def test_deep_recursion_batched_launches():
    """Frames whose deep levels exceed one launch's buffer are rendered in chunk batches
    (render.hip launch_full): 16 tiles x 64 lanes x 284 levels x 128 B = 37 MB per chunk,
    so a 40 MB cap gives one chunk per launch.  The result must not depend on the batching."""
    _compare(_mirror_corridor(300, 128, 64), chunk_first=1, chunk_step=2, options={"deep_cap_mb": 40})


def test_deep_recursion_refused_past_the_buffer():
    eng = M.RayTracerEngine(_mirror_corridor(300, 128, 64))
    eng.set_option("deep_cap_mb", 1)
    with pytest.raises(M.RenderError) as e:
        eng.render(0)
    assert e.value.code == A.RT_ERR_UNSUPPORTED
    eng.close()


# ------------------------------------------------ compacted bounce render (render.hip k_bounce)
def _rough_mirror_scene(w=128, h=96):
    sc = _primitives_scene(w, h)
    sc.materials.append(M.Material(ambient=(0.05, 0.05, 0.05), diffuse=(0.2, 0.2, 0.2), specular=(0.5, 0.5, 0.5),
                                   phong=40.0, mirror=(0.8, 0.8, 0.8), roughness=0.05, type="mirror"))
    sc.objects[3].material = "6"                       # rough mirror: PCG32 draws per bounce level
    return sc


@pytest.mark.parametrize("queue,tail", [(0, 0), (1, 0), (1, 1), (1, 2)])
def test_queued_bounces_against_the_oracle(queue, tail):
    """Mirror/conductor scenes through the compacted bounce render (option queue = 1, the default:
    primary pass + one k_bounce launch per level, rays resolved backward through their queue
    records; with queue_tail = t the levels >= t traced depth-first in one k_bounce_tail launch)
    and through the bounce megakernel (0): all equal the oracle's recursion
    (Object+Extension.swift:189-206, 252-283).  Covers the general walk (a transformed
    instance), rough mirrors, spp 3 (one traced sample divided by 3), the unified walk with 15
    queue levels, chunk selections, and several replicas."""
    opt = {"queue": queue, "queue_tail": tail}
    sc = _rough_mirror_scene()
    st = _compare(sc, options=opt)
    assert st.secondary_rays > 0
    sc.cameras[0].num_samples = 3
    _compare(sc, options=opt)
    st = _compare(_mirror_corridor(15, 48, 36), options=opt)
    assert st.secondary_rays > 10 * 48 * 36 // 2
    _compare(_mirror_corridor(12, 48, 36), chunk_first=1, chunk_step=3, options=opt)
    # 3 chunks -> rt_render_ex's two staged launches of different sizes share one queue arena
    _compare(_mirror_corridor(8, 64, 40), chunk_first=0, chunk_step=2, options=opt)
    sc = _mirror_corridor(8, 56, 40)
    ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    eng = M.RayTracerEngine(sc, devices=[0, 0, 0])
    eng.set_option("queue", queue)
    eng.set_option("queue_tail", tail)
    for _ in range(2):                                 # queue words must be back at zero
        rgb, rgba, st = eng.render_rows(0, 0, 1, True)
        assert float(np.abs(rgb - ref).max()) <= TOL and np.array_equal(rgba, ref8)
        assert st.secondary_rays == ost.secondary_rays
    eng.close()
