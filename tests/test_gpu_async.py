"""Renders in flight: rt_render_submit / rt_render_wait (the reference's render is async,
RayTracer.swift:115-131, 137-205; bench.py keeps RT_MAX_IN_FLIGHT frames in flight).

Each submitted render must deliver exactly the image and counts the synchronous rt_render_ex
delivers (which is itself checked against the oracle, test_gpu_frames.py / test_gpu_parity.py),
whatever else is in flight: different cameras and chunk selections at once, waits out of order,
several replicas, and full trace() renders (dielectrics, area lights) on their slot streams.
Errors: too many in flight (RT_ERR_BUSY), unknown or repeated tickets, pageable outputs."""
import copy

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import _abi as A
from myraytracer_amd import scenes
import oracle

pytestmark = pytest.mark.gpu


def _sync(eng, cam, first, step, H, W):
    rgb = M.pinned_array((H, W, 3), np.float64)
    rgba = M.pinned_array((H, W, 4), np.uint8)
    rgb.fill(-1.0)
    rgba.fill(0)
    st = eng.render_into(cam, first, step, rgb=rgb, rgba=rgba, frame_layout=True)
    return rgb, rgba, st


def _two_camera_c2(w=200, h=150):
    sc = scenes.scaled(scenes.scene_c2(inline=True), w, h)
    c2 = copy.deepcopy(sc.cameras[0])
    c2.position = (1.5, 1.0, 3.5)
    sc.cameras.append(c2)
    return sc


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_in_flight_renders_match_synchronous_renders(devices):
    sc = _two_camera_c2()
    W, H = sc.cameras[0].image_resolution
    eng = M.RayTracerEngine(sc, devices=devices)
    jobs = [(0, 0, 1), (1, 0, 1), (0, 1, 3), (1, 2, 2)]      # (camera, chunk_first, chunk_step)
    want = [_sync(eng, *j, H, W) for j in jobs]
    outs = [(M.pinned_array((H, W, 3), np.float64), M.pinned_array((H, W, 4), np.uint8)) for _ in jobs]
    for rgb, rgba in outs:
        rgb.fill(-1.0)
        rgba.fill(0)
    # every other render asks for kernel timing (RT_RENDER_KERNEL_TIME)
    tickets = [eng.submit_into(c, f, s, rgb=o[0], rgba=o[1], frame_layout=True, kernel_time=(k % 2 == 0))
               for k, ((c, f, s), o) in enumerate(zip(jobs, outs))]
    assert len(set(tickets)) == len(tickets)
    for k in (2, 0, 3, 1):                                    # out of order
        st = eng.wait(tickets[k])
        rgb, rgba, ws = want[k]
        assert np.array_equal(outs[k][0], rgb) and np.array_equal(outs[k][1], rgba)
        assert (st.primary_rays, st.shadow_rays, st.shadow_rays_traced) == \
               (ws.primary_rays, ws.shadow_rays, ws.shadow_rays_traced)
        assert st.milliseconds > 0
        assert (st.kernel_ms > 0) if k % 2 == 0 else (st.kernel_ms == 0)
    eng.close()


def test_pipelined_frames_against_the_oracle():
    """Many frames in flight through one engine (bench.py's loop), each checked against the
    oracle: ring of RT_MAX_IN_FLIGHT framebuffers, wait for the oldest before each submit."""
    sc = scenes.scaled(scenes.scene_c2(inline=True), 160, 120)
    ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    eng = M.RayTracerEngine(sc)
    Q = A.RT_MAX_IN_FLIGHT
    fbs = [M.pinned_array((120, 160, 4), np.uint8) for _ in range(Q)]
    pend = []
    for k in range(3 * Q + 1):
        if len(pend) == Q:
            kk, t = pend.pop(0)
            st = eng.wait(t)
            assert np.array_equal(fbs[kk % Q], ref8) and st.shadow_rays == ost.shadow_rays
        fbs[k % Q].fill(0)
        pend.append((k, eng.submit_into(0, 0, 1, rgba=fbs[k % Q], frame_layout=True)))
    for kk, t in pend:
        eng.wait(t)
        assert np.array_equal(fbs[kk % Q], ref8)
    eng.close()


@pytest.mark.parametrize("full_flights", [0, 2, 4])
def test_full_trace_renders_in_flight(full_flights):
    """Dielectrics / area lights take the full trace() passes (render_full.h), whose scratch
    (event counts, jitter prefixes, hit log, node records) belongs to a stream: submitted renders
    take slot q % full_flights's stream and scratch (render option), so up to that many overlap (0: all on
    the replica's stream, in order).  Two cameras, chunk selections and glass at once, waits in
    a ring; every frame equals rt_render_ex's."""
    from test_gpu_features import _area_scene
    sc = _area_scene(96, 64)                                 # area lights (render_full)
    sc.objects[3].material = "3"                             # + glass
    c2 = copy.deepcopy(sc.cameras[0])
    c2.position = (1.0, 1.5, 5.0)
    sc.cameras.append(c2)
    W, H = sc.cameras[0].image_resolution
    eng = M.RayTracerEngine(sc)
    eng.set_option("full_flights", full_flights)
    jobs = [(0, 0, 1), (1, 0, 1), (0, 1, 3), (1, 2, 2)]
    want = [_sync(eng, *j, H, W) for j in jobs]
    Q = 6
    outs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]
    pend = []
    for k in range(3 * len(jobs)):
        if len(pend) == Q:
            kk, t = pend.pop(0)
            st = eng.wait(t)
            assert np.array_equal(outs[kk % Q], want[kk % len(jobs)][1])
            assert st.shadow_rays == want[kk % len(jobs)][2].shadow_rays
        outs[k % Q].fill(0)
        pend.append((k, eng.submit_into(*jobs[k % len(jobs)], rgba=outs[k % Q], frame_layout=True)))
    for kk, t in pend:
        st = eng.wait(t)
        assert np.array_equal(outs[kk % Q], want[kk % len(jobs)][1])
        assert st.secondary_rays == want[kk % len(jobs)][2].secondary_rays
    eng.close()


def test_submit_errors():
    sc = scenes.scaled(scenes.scene_c2(inline=True), 64, 48)
    eng = M.RayTracerEngine(sc)
    Q = A.RT_MAX_IN_FLIGHT
    outs = [M.pinned_array((48, 64, 4), np.uint8) for _ in range(Q + 1)]
    ts = [eng.submit_into(0, 0, 1, rgba=outs[k], frame_layout=True) for k in range(Q)]
    with pytest.raises(M.RenderError) as e:                  # one too many in flight
        eng.submit_into(0, 0, 1, rgba=outs[Q], frame_layout=True)
    assert e.value.code == A.RT_ERR_BUSY
    with pytest.raises(M.RenderError):                       # never submitted
        eng.wait(ts[-1] + 100)
    eng.wait(ts[1])
    with pytest.raises(M.RenderError):                       # already waited for
        eng.wait(ts[1])
    with pytest.raises(M.RenderError) as e:                  # pageable output
        eng.submit_into(0, 0, 1, rgba=np.zeros((48, 64, 4), np.uint8), frame_layout=True)
    assert e.value.code == A.RT_ERR_INVALID_ARG
    for t in (ts[0], ts[2], ts[3]):
        eng.wait(t)
    # a slot freed by a wait takes the next submit; rt_render_ex still works meanwhile
    t = eng.submit_into(0, 0, 1, rgba=outs[Q], frame_layout=True)
    rgb, rgba, _ = _sync(eng, 0, 0, 1, 48, 64)
    eng.wait(t)
    assert np.array_equal(outs[Q], rgba)
    eng.close()


def test_failed_replica_launch_drains_and_frees_the_slot():
    """A launch that fails on replica k > 0 (forced: option debug_fail_replica) must not leave
    replicas 0..k-1 writing into the caller's buffers behind an error: they are drained before
    rt_render_submit returns, and the slot is free again (every slot still takes a render)."""
    sc = scenes.scaled(scenes.scene_c2(inline=True), 96, 72)
    W, H = sc.cameras[0].image_resolution
    eng = M.RayTracerEngine(sc, devices=[0, 0, 0])
    want = _sync(eng, 0, 0, 1, H, W)
    out = M.pinned_array((H, W, 4), np.uint8)
    out.fill(0)
    eng.set_unsafe_option("debug_fail_replica", 1)
    with pytest.raises(M.RenderError) as e:
        eng.submit_into(0, 0, 1, rgba=out, frame_layout=True)
    assert e.value.code == A.RT_ERR_DEVICE and "injected" in str(e.value)
    with pytest.raises(M.RenderError) as e:                  # rt_render_ex shares the path
        eng.render_into(0, 0, 1, rgba=out, frame_layout=True)
    assert e.value.code == A.RT_ERR_DEVICE
    # replica 0's rows (chunks 0, 3, 6, ...) were rendered and drained; nothing else was written
    rows = np.zeros(H, bool)
    for c in range(0, (H + 7) // 8, 3):
        rows[8 * c: 8 * c + 8] = True
    snap = out.copy()
    assert np.array_equal(snap[rows], want[1][rows]) and np.all(snap[~rows] == 0)
    eng.set_unsafe_option("debug_fail_replica", -1)
    outs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(A.RT_MAX_IN_FLIGHT)]
    ts = [eng.submit_into(0, 0, 1, rgba=o, frame_layout=True) for o in outs]
    for t, o in zip(ts, outs):
        eng.wait(t)
        assert np.array_equal(o, want[1])
    assert np.array_equal(out, snap)                         # no late writes from the failed submits
    eng.close()


def test_concurrent_waits_on_one_ticket():
    """Two threads waiting on the same ticket: exactly one gets the render's stats, the other
    an error (it must never return the counts of a later render reusing the slot)."""
    import threading
    sc = scenes.scaled(scenes.scene_c2(inline=True), 400, 300)
    W, H = sc.cameras[0].image_resolution
    eng = M.RayTracerEngine(sc)
    want = _sync(eng, 0, 0, 1, H, W)[2]
    for _ in range(5):
        out = M.pinned_array((H, W, 4), np.uint8)
        t = eng.submit_into(0, 0, 1, rgba=out, frame_layout=True)
        res = []

        def waiter():
            try:
                res.append(("ok", eng.wait(t)))
            except M.RenderError as e:
                res.append(("err", e.code))
        th = [threading.Thread(target=waiter) for _ in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        oks = [r for k, r in res if k == "ok"]
        assert len(oks) == 1 and len(res) == 2
        assert oks[0].shadow_rays == want.shadow_rays
        assert [r for k, r in res if k == "err"] == [A.RT_ERR_INVALID_ARG]
    eng.close()


@pytest.mark.parametrize("queue,tail", [(0, 0), (1, 0), (1, 2)])
def test_pipelined_mirror_frames_against_the_oracle(queue, tail):
    """Mirror frames in flight (each slot has its own bounce queues and counters): every frame
    equals the oracle and carries the oracle's secondary-ray count."""
    from test_gpu_features import _mirror_corridor
    sc = _mirror_corridor(6, 80, 56)
    ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    eng = M.RayTracerEngine(sc)
    eng.set_option("queue", queue)
    eng.set_option("queue_tail", tail)
    Q = A.RT_MAX_IN_FLIGHT
    fbs = [M.pinned_array((56, 80, 4), np.uint8) for _ in range(Q)]
    pend = []
    for k in range(2 * Q + 3):
        if len(pend) == Q:
            kk, t = pend.pop(0)
            st = eng.wait(t)
            assert np.array_equal(fbs[kk % Q], ref8)
            assert (st.shadow_rays, st.secondary_rays) == (ost.shadow_rays, ost.secondary_rays)
        fbs[k % Q].fill(0)
        pend.append((k, eng.submit_into(0, 0, 1, rgba=fbs[k % Q], frame_layout=True)))
    for kk, t in pend:
        eng.wait(t)
        assert np.array_equal(fbs[kk % Q], ref8)
    eng.close()


def _chunk_rows(H, first, step):
    rows = np.zeros(H, bool)
    for c in range(first, (H + 7) // 8, step):
        rows[8 * c: 8 * c + 8] = True
    return rows


def test_scratch_growth_beside_renders_in_flight():
    """Scratch grows while other renders are in flight (the race class of round 4's
    undelivered mirror pixels): the compacted bounce render's queues of every in-flight slot grow
    three times (a quarter, half, then all of the chunks) while the other slots' renders run, and
    two device renders on one stream grow the device path's queues back to back with no host
    synchronisation between them.  Grown buffers' predecessors are retired, not freed, and the new
    ones are zeroed on the growing render's stream (render.hip retire / queue_arena).  Every frame
    equals the oracle on its selected rows."""
    import torch
    from test_gpu_features import _mirror_corridor
    sc = _mirror_corridor(4, 96, 64)
    W, H = 96, 64
    ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    eng = M.RayTracerEngine(sc)
    assert eng.get_option("queue") == 1
    Q = A.RT_MAX_IN_FLIGHT
    sels = [(k % 4, 4) for k in range(Q)] + [(k % 2, 2) for k in range(Q)] + [(0, 1)] * (Q + 3)
    fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]
    pend = []

    def check(kk, t):
        eng.wait(t)
        rows = _chunk_rows(H, *sels[kk])
        got = fbs[kk % Q]
        assert np.array_equal(got[rows], ref8[rows]), f"frame {kk} (chunks {sels[kk]}) differs"
        assert not got[~rows].any()

    for k, (first, step) in enumerate(sels):
        if len(pend) == Q:
            check(*pend.pop(0))
        fbs[k % Q].fill(0)
        pend.append((k, eng.submit_into(0, first, step, rgba=fbs[k % Q], frame_layout=True)))
    for kk, t in pend:
        check(kk, t)
    # device path: two renders on one stream, the second growing the queues the first still uses
    s = torch.cuda.Stream()
    small = torch.full((H // 4 + 8, W, 3), -1.0, dtype=torch.float64, device="cuda")
    full = torch.full((H, W, 3), -1.0, dtype=torch.float64, device="cuda")
    eng.render_device(small.data_ptr(), 0, 1, 4, stream=s.cuda_stream)
    eng.render_device(full.data_ptr(), 0, 0, 1, stream=s.cuda_stream)
    s.synchronize()
    assert float(np.abs(full.cpu().numpy() - ref).max()) <= 1e-5
    rows = _chunk_rows(H, 1, 4)
    assert float(np.abs(small.cpu().numpy()[: rows.sum()] - ref[rows]).max()) <= 1e-5
    assert eng.info().scratch_bytes > 0
    eng.close()


def _mirror_ball(w=160, h=120, depth=3):
    """A diffuse floor with one mirror sphere over it: a minority of the pixels reflect, and some
    of their reflected rays hit the sphere's own floor image and stop."""
    mats = [M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.6, 0.7, 0.5), specular=(0.3, 0.3, 0.3), phong=16.0),
            M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.2, 0.2, 0.2), specular=(0.4, 0.4, 0.4), phong=24.0,
                       mirror=(0.7, 0.7, 0.7), type="mirror")]
    floor = M.Mesh(id=1, material="1", positions=np.array([[-8, 0, 8], [8, 0, 8], [8, 0, -8], [-8, 0, -8]], np.float64),
                   indices=np.array([[1, 2, 3], [1, 3, 4]], np.int32), shading_mode="flat")
    cam = M.Camera(position=(0.0, 3.0, 7.0), gaze_point=(0.0, 0.8, 0.0), up=(0.0, 1.0, 0.0), fovy=45.0,
                   image_resolution=(w, h))
    return M.Scene(cameras=[cam], materials=mats,
                   objects=[floor, M.Sphere(center=(0.4, 1.0, 0.0), radius=1.0, material="2"),
                            M.Sphere(center=(-1.6, 0.6, 1.2), radius=0.6, material="2")],
                   point_lights=[M.PointLight((3.0, 6.0, 4.0), (600.0, 600.0, 600.0))],
                   ambient_light=(15.0, 15.0, 15.0), background_color=(40.0, 60.0, 90.0),
                   shadow_ray_epsilon=1e-3, intersection_test_epsilon=1e-6, max_recursion_depth=depth)


@pytest.mark.parametrize("scene", ["ball", "corridor"])
def test_bounce_queues_hold_only_the_rays(scene):
    """Compacted bounce render, records compacted per level: a level holds only its
    rays, so the 16 in-flight slots' arenas are sized by the rays, not by levels x pixels x 128 B.
    Each slot's arena starts at the replica's measured need (1/16 of the worst case before any is
    known): the corridor, where nearly every pixel reflects, overflows that first guess and its
    frame is rendered again on a grown arena (render.hip wait_impl).  Every frame of three
    pipelined rounds equals the oracle, and the scratch stops growing after the first round
    (retired buffers are freed once nothing is in flight)."""
    from test_gpu_features import _mirror_corridor
    sc = _mirror_ball() if scene == "ball" else _mirror_corridor(4, 96, 64)
    W, H = sc.cameras[0].image_resolution
    ref, ref8, ost = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
    eng = M.RayTracerEngine(sc)
    assert eng.get_option("queue") == 1
    Q = A.RT_MAX_IN_FLIGHT
    fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(Q)]
    submit, wait = eng.frame_pipeline(0, 0, 1, fbs, frame_layout=True)
    scratch = []
    for rnd in range(3):
        for fb in fbs:
            fb.fill(0)
        ts = [submit(k) for k in range(Q)]
        for k, t in enumerate(ts):
            st = wait(t)
            assert np.array_equal(fbs[k], ref8), f"round {rnd} frame {k} differs"
            assert st.secondary_rays == ost.secondary_rays and st.shadow_rays == ost.shadow_rays
        scratch.append(eng.info().scratch_bytes)
    levels = sc.max_recursion_depth
    per_pixel_layout = Q * levels * W * H * 128            # the round-5 arenas: a record per pixel and level
    print(f"{scene}: scratch {scratch} B; per-pixel layout {per_pixel_layout} B; "
          f"secondary rays {ost.secondary_rays} of {levels * W * H} slots")
    assert scratch[1] == scratch[2] and scratch[0] >= scratch[1]
    if scene == "ball":
        assert scratch[2] < per_pixel_layout / 4
    eng.close()
