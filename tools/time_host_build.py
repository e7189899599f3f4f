import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C, sys
from myraytracer_amd import scenes, _abi as A
from myraytracer_amd.engine import load_library
sc = scenes.scene_c5(path_dir="scenes_cache")
lib = load_library(); pk = sc.to_desc()
hs = (C.c_uint64 * 256)(); n = C.c_int32(); info = A.rt_scene_info()
rc = lib.rt_debug_host_build(pk.ptr, hs, 256, C.byref(n), C.byref(info))
