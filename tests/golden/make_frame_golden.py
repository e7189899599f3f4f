#!/usr/bin/env python3
"""Freeze the CPU oracle's framebuffers (test infrastructure; VERDICT r1 "freeze the oracle").

For each scene of frame_scenes.py: the geometry goes to frames/<name>.npz (float32 positions,
int32 indices) and the oracle's render (oracle/rt_oracle.cpp, the restatement of the reference's
Renderer.render + trace(), Object+Extension.swift:52-379) to frames/expected.json:
  rgb_sha256    SHA-256 of the FP64 framebuffer bytes (H, W, 3) little-endian
  rgba8_sha256  SHA-256 of the RGBA8 image (RayTracer.swift:186-195)
  samples       256 seeded pixel positions with the three doubles as IEEE hex
  rays          primary / shadow / secondary ray counts
tests/test_golden_frames.py re-renders with the oracle (bit-exact against the hashes) and with
the GPU (within the 1e-5 parity bar, exact RGBA8).  Regenerate only when the oracle is meant to
change:  python tests/golden/make_frame_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import frame_scenes as FS  # noqa: E402
import oracle  # noqa: E402


def frame_record(rgb, rgba, st, seed):
    H, W = rgb.shape[:2]
    rng = np.random.RandomState(seed)
    idx = sorted(set(zip(rng.randint(0, H, 300).tolist(), rng.randint(0, W, 300).tolist())))[:256]
    return {"shape": [H, W],
            "rgb_sha256": hashlib.sha256(np.ascontiguousarray(rgb, dtype="<f8").tobytes()).hexdigest(),
            "rgba8_sha256": hashlib.sha256(np.ascontiguousarray(rgba).tobytes()).hexdigest(),
            "samples": [[r, c] + [float(v).hex() for v in rgb[r, c]] for r, c in idx],
            "rays": {"primary": int(st.primary_rays), "shadow": int(st.shadow_rays),
                     "secondary": int(st.secondary_rays)}}


def main():
    os.makedirs(FS.FRAMES, exist_ok=True)
    out = {}
    for k, name in enumerate(FS.NAMES):
        if name != "c1":
            P, I = FS.geometry(name)
            np.savez(os.path.join(FS.FRAMES, f"{name}.npz"), positions=P, indices=I)
        sc = FS.scene(name)
        rgb, rgba, st = oracle.OracleScene(sc).render(0, threads=0, rgba=True)
        out[name] = frame_record(rgb, rgba, st, 1000 + k)
        print(name, rgb.shape, out[name]["rgb_sha256"][:16], out[name]["rays"])
    with open(os.path.join(FS.FRAMES, "expected.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
