#!/usr/bin/env python3
"""Generate PLY golden vectors from the REFERENCE's own CPly (miniply + wrapper).

Inputs (tests/golden/ply/*.ply) are small synthetic files written here; expected
outputs (tests/golden/ply/*.json) are what the reference's PLYLoader.load
(Sources/RayTracer/Helpers/PLYReader.swift:54-210) gets from CPly, driven through
oracle.RefCPly against oracle/_ref/libcply_ref.so (built by oracle/build_ref.sh from
/root/reference/Sources/CPly).  Run in the build container only:

    bash oracle/build_ref.sh && python tests/golden/make_ply_golden.py
"""
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
OUT = os.path.join(HERE, "ply")

TYPES = {"char": "b", "uchar": "B", "short": "h", "ushort": "H", "int": "i", "uint": "I", "float": "f",
         "double": "d"}


def write(name, fmt, vprops, verts, face_ctype, face_itype, faces, extra_header="", face_extra=None):
    """vprops: list of (type, name); verts: list of tuples; faces: list of index lists."""
    lines = ["ply", f"format {fmt} 1.0", "comment golden vector for the PLY reader", "obj_info generated"]
    if extra_header:
        lines.append(extra_header)
    lines.append(f"element vertex {len(verts)}")
    lines += [f"property {t} {n}" for t, n in vprops]
    lines.append(f"element face {len(faces)}")
    lines.append(f"property list {face_ctype} {face_itype} vertex_indices")
    if face_extra:
        lines.append(f"property {face_extra[0]} {face_extra[1]}")
    lines.append("end_header")
    path = os.path.join(OUT, name + ".ply")
    with open(path, "wb") as fh:
        fh.write(("\n".join(lines) + "\n").encode())
        if fmt == "ascii":
            for v in verts:
                fh.write((" ".join(str(x) for x in v) + "\n").encode())
            for f in faces:
                row = [len(f)] + list(f) + ([7] if face_extra else [])
                fh.write((" ".join(str(x) for x in row) + "\n").encode())
        else:
            e = "<" if fmt == "binary_little_endian" else ">"
            for v in verts:
                for (t, _), x in zip(vprops, v):
                    fh.write(struct.pack(e + TYPES[t], x))
            for f in faces:
                fh.write(struct.pack(e + TYPES[face_ctype], len(f)))
                for x in f:
                    fh.write(struct.pack(e + TYPES[face_itype], x))
                if face_extra:
                    fh.write(struct.pack(e + TYPES[face_extra[0]], 7))
    return path


def cases():
    xyz = [("float", "x"), ("float", "y"), ("float", "z")]
    quad_v = [(0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (1.0, 1.0, 0.0), (0.0, 1.0, 0.0), (0.5, 1.7, 0.25)]
    rng = np.random.RandomState(3)
    grid = [tuple(float(np.float32(c)) for c in rng.uniform(-2, 2, 3)) for _ in range(12)]
    tris = [[0, 1, 2], [2, 3, 0], [1, 4, 2]]
    yield write("tri_binary_le", "binary_little_endian", xyz, quad_v, "uchar", "int", tris)
    yield write("tri_binary_be", "binary_big_endian", xyz, quad_v, "uchar", "int", tris)
    yield write("tri_ascii", "ascii", xyz, [(0.125, -0.5, 3.25), (1.1, 0.3, 2.7), (0.1, 0.7e-1, 1e2), (2.5e-3, -7.25, 0.3)],
                "uchar", "int", [[0, 1, 2], [1, 3, 2]])
    yield write("quad_mix_le", "binary_little_endian", xyz, quad_v, "uchar", "int", [[0, 1, 2, 3], [1, 4, 2]])
    yield write("quad_uint_ushort", "binary_little_endian", xyz, quad_v, "uchar", "uint", [[0, 1, 2, 3]])
    yield write("quad_ushort_idx", "binary_big_endian", xyz, quad_v, "uchar", "ushort", [[3, 2, 1, 0], [0, 1, 4]])
    # pentagon / hexagon faces: ear clipping in float32 (miniply.cpp:1987-2055)
    pent = [(np.cos(a), np.sin(a), 0.1 * k) for k, a in enumerate(np.linspace(0, 2 * np.pi, 6)[:5])]
    pent = [tuple(float(np.float32(c)) for c in p) for p in pent]
    yield write("pentagon_last", "binary_little_endian", xyz, pent, "uchar", "int", [[0, 1, 2], [0, 1, 2, 3, 4]])
    hexv = [(np.cos(a) * (1 + 0.3 * (k % 2)), np.sin(a), 0.0) for k, a in enumerate(np.linspace(0, 2 * np.pi, 7)[:6])]
    hexv = [tuple(float(np.float32(c)) for c in p) for p in hexv]
    yield write("hexagon_first", "binary_little_endian", xyz, hexv, "uchar", "int", [[0, 1, 2, 3, 4, 5], [0, 2, 4], [1, 3, 5]])
    # normals + texcoords; doubles; ints as coordinates
    xyzn = xyz + [("float", "nx"), ("float", "ny"), ("float", "nz"), ("float", "u"), ("float", "v")]
    vn = [g + (0.3, 0.4 + i * 0.1, 1.0, 0.25 * i, 1.0 - 0.1 * i) for i, g in enumerate(grid[:4])]
    yield write("normals_uv", "binary_little_endian", xyzn, vn, "uchar", "int", [[0, 1, 2], [0, 2, 3]])
    xyzd = [("double", "x"), ("double", "y"), ("double", "z")]
    yield write("double_coords", "binary_little_endian", xyzd, [(0.1, 0.2, 0.3), (1.0 / 3, -2.0 / 7, 1e-9), (5.5, 6.25, -1.125)],
                "uchar", "int", [[0, 1, 2]])
    xyzi = [("int", "x"), ("short", "y"), ("uchar", "z")]
    yield write("int_coords", "ascii", xyzi, [(1, -2, 3), (40000, 5, 255), (-7, 32000, 0)], "uchar", "int", [[2, 1, 0]])
    # extra per-face property after the list; extra vertex property in between
    xyzq = [("float", "x"), ("float", "confidence"), ("float", "y"), ("float", "z")]
    yield write("extra_props", "binary_little_endian", xyzq, [(0, 9, 0, 0), (1, 9, 0, 0), (0, 9, 1, 0)], "uchar", "int",
                [[0, 1, 2]], face_extra=("uchar", "flags"))
    yield write("ascii_quads", "ascii", xyz, quad_v, "uchar", "int", [[0, 1, 2, 3], [0, 1, 4]])
    # degenerate/edge: faces with < 3 vertices mixed in
    yield write("short_faces", "binary_little_endian", xyz, quad_v, "uchar", "int", [[0, 1], [0, 1, 2], [3]])
    # no face element -> faceDataMissing
    p = os.path.join(OUT, "no_faces.ply")
    with open(p, "w") as fh:
        fh.write("ply\nformat ascii 1.0\nelement vertex 1\nproperty float x\nproperty float y\nproperty float z\nend_header\n0 0 0\n")
    yield p
    # corrupted header -> corrupted
    p = os.path.join(OUT, "corrupt_header.ply")
    with open(p, "w") as fh:
        fh.write("ply\nformat banana 1.0\nend_header\n")
    yield p


def enc(x):
    if x is None:
        return None
    a = np.asarray(x)
    if a.dtype.kind == "f":
        return [float(v).hex() for v in a.reshape(-1).astype(np.float64)]
    return [int(v) for v in a.reshape(-1)]


def main():
    import oracle
    os.makedirs(OUT, exist_ok=True)
    ref = oracle.RefCPly()
    for path in cases():
        name = os.path.splitext(os.path.basename(path))[0]
        try:
            m = ref.load(path)
            rec = {"ok": True, "positions": enc(m["positions"]), "normals": enc(m["normals"]),
                   "texcoords": enc(m["texcoords"]), "indices": enc(m["indices"])}
        except ValueError as e:
            rec = {"ok": False, "error": str(e)}
        with open(os.path.join(OUT, name + ".json"), "w") as fh:
            json.dump(rec, fh, indent=0)
        print(name, rec.get("error", f"{len(rec.get('indices') or [])} indices"))
    missing = os.path.join(OUT, "does_not_exist.ply")
    try:
        ref.load(missing)
        rec = {"ok": True}
    except ValueError as e:
        rec = {"ok": False, "error": str(e)}
    with open(os.path.join(OUT, "missing_file.json"), "w") as fh:
        json.dump(rec, fh)
    print("missing_file", rec)


if __name__ == "__main__":
    main()
