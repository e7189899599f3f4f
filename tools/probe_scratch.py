"""Device scratch a scene holds (rt_scene_info.scratch_bytes) step by step through the compacted
bounce render: after creation, one synchronous frame, the 16-deep pipeline's first pass and three
pipelined rounds (tests/test_gpu_async.py scenes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np

import myraytracer_amd as M
from myraytracer_amd import _abi as A

from test_gpu_async import _mirror_ball
from test_gpu_features import _mirror_corridor

for name, sc in (("corridor", _mirror_corridor(4, 96, 64)), ("ball", _mirror_ball())):
    W, H = sc.cameras[0].image_resolution
    eng = M.RayTracerEngine(sc)
    print(name, "created", eng.info().scratch_bytes, flush=True)
    fb = M.pinned_array((H, W, 4), np.uint8)
    eng.render_into(0, 0, 1, None, fb, True)
    print(name, "one frame", eng.info().scratch_bytes, flush=True)
    fbs = [M.pinned_array((H, W, 4), np.uint8) for _ in range(A.RT_MAX_IN_FLIGHT)]
    submit, wait = eng.frame_pipeline(0, 0, 1, fbs, frame_layout=True)
    print(name, "pipeline first pass", eng.info().scratch_bytes, flush=True)
    for r in range(3):
        ts = [submit(k) for k in range(len(fbs))]
        for t in ts:
            wait(t)
        print(name, "round", r, eng.info().scratch_bytes, flush=True)
    eng.close()
