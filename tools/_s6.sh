G="python -u bench.py --config c3g --steps 30 --warmup 3 --no-cpu-baseline --no-side-paths"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
tools/gpu_session.sh \
 "suite|600|$T tests -m gpu" \
 "g_p4|200|$G" \
 "g_pos|200|MYRT_LIB=build_variants/libmyrt_pos.so $G" \
 "g_p4b|200|$G" \
 "g_posb|200|MYRT_LIB=build_variants/libmyrt_pos.so $G"
for f in gpurun_out/g_p*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"one_frame_ms": [0-9.]*' $f)"; done
