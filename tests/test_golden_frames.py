"""Frozen oracle framebuffers (tests/golden/frames/, made by tests/golden/make_frame_golden.py).

The render oracle cannot be pinned to the Swift reference (no toolchain, no fixtures: SURVEY.md
§8c), so its output is frozen: any later edit of oracle/rt_oracle.cpp that changes a single bit
of these frames fails here.  The scenes cover C1, a ~5k-triangle smooth mesh with two point
lights, and a mirror mesh + glass sphere + ground under a point light and two area lights at
4 spp (render_full: dielectric recursion, the per-chunk jitterIndex scan).
CPU: the oracle against the hashes, bit-exact.  GPU: the product against the samples (1e-5,
the parity bar) and the RGBA8 hash (exact)."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import frame_scenes as FS  # noqa: E402
import myraytracer_amd as M  # noqa: E402
import oracle  # noqa: E402

with open(os.path.join(FS.FRAMES, "expected.json")) as _fh:
    EXPECTED = json.load(_fh)


def _sha(a, dt=None):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=dt).tobytes()).hexdigest()


@pytest.mark.parametrize("name", FS.NAMES)
def test_oracle_reproduces_the_frozen_frame(name):
    exp = EXPECTED[name]
    rgb, rgba, st = oracle.OracleScene(FS.scene(name)).render(0, threads=0, rgba=True)
    assert list(rgb.shape[:2]) == exp["shape"]
    assert (st.primary_rays, st.shadow_rays, st.secondary_rays) == tuple(exp["rays"][k] for k in
                                                                        ("primary", "shadow", "secondary"))
    for r, c, *hx in exp["samples"]:
        assert [float(v).hex() for v in rgb[r, c]] == hx, (r, c)
    assert _sha(rgb, "<f8") == exp["rgb_sha256"]
    assert _sha(rgba) == exp["rgba8_sha256"]


def test_frozen_frames_are_not_trivial():
    for name in FS.NAMES:
        vals = np.array([[float.fromhex(h) for h in s[2:]] for s in EXPECTED[name]["samples"]])
        assert len(np.unique(vals.round(6), axis=0)) > 20, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", FS.NAMES)
def test_gpu_matches_the_frozen_frame(name):
    exp = EXPECTED[name]
    eng = M.RayTracerEngine(FS.scene(name))
    res = eng.render(0)
    for r, c, *hx in exp["samples"]:
        want = np.array([float.fromhex(h) for h in hx])
        assert float(np.abs(res.rgb[r, c] - want).max()) <= 1e-5, (r, c, res.rgb[r, c], want)
    assert _sha(res.rgba8) == exp["rgba8_sha256"]
    st = res.stats
    assert (st.primary_rays, st.shadow_rays, st.secondary_rays) == tuple(exp["rays"][k] for k in
                                                                        ("primary", "shadow", "secondary"))
    eng.close()
