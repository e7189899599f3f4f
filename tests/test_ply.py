"""Product PLY reader (libmyrt.so rt_ply_load) vs golden vectors produced by the
reference's own CPly (tests/golden/make_ply_golden.py).  Bit-exact for every array."""
import glob
import json
import os

import numpy as np
import pytest

import myraytracer_amd as M
from myraytracer_amd import scenes

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ply")
CASES = sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLD, "*.ply")))


def dec(v):
    if v is None:
        return None
    if v and isinstance(v[0], str):
        return np.array([float.fromhex(x) for x in v])
    return np.array(v, dtype=np.int64)


@pytest.mark.parametrize("name", CASES)
def test_ply_matches_reference_cply(name):
    with open(os.path.join(GOLD, name + ".json")) as fh:
        g = json.load(fh)
    path = os.path.join(GOLD, name + ".ply")
    if not g["ok"]:
        with pytest.raises(M.RenderError) as e:
            M.ply_load(path)
        assert e.value.code == -40
        return
    m = M.ply_load(path)
    assert np.array_equal(m["positions"].reshape(-1), dec(g["positions"]))
    if g["normals"] is None:
        assert m["normals"] is None
    else:
        assert np.array_equal(m["normals"].reshape(-1), dec(g["normals"]))
    if g["texcoords"] is None:
        assert m["texcoords"] is None
    else:
        assert np.array_equal(m["texcoords"].reshape(-1).astype(np.float64), dec(g["texcoords"]))
    assert np.array_equal(np.asarray(m["indices"]).reshape(-1), dec(g["indices"]))


def test_missing_file_is_an_error():
    with pytest.raises(M.RenderError) as e:
        M.ply_load(os.path.join(GOLD, "does_not_exist.ply"))
    assert e.value.code == -40


@pytest.mark.parametrize("fmt", ["binary_little_endian", "binary_big_endian", "ascii"])
def test_generated_scene_roundtrip(tmp_path, fmt):
    pos, faces = scenes.geometry_c2(segments=24, rings=12)
    p = str(tmp_path / f"c2_{fmt}.ply")
    scenes.write_ply(p, pos, faces, fmt=fmt)
    m = M.ply_load(p)
    assert np.array_equal(m["positions"], pos.astype(np.float32).astype(np.float64))
    assert np.array_equal(m["indices"], faces)
