G="python -u bench.py --config c3g --steps 30 --warmup 3 --no-cpu-baseline --no-side-paths"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
tools/gpu_session.sh \
 "lt|400|$T tests/test_gpu_features.py tests/test_gpu_async.py tests/test_golden_frames.py -k 'area or dielectric or full_trace or glass'" \
 "g_new|200|$G" \
 "g_pos|200|MYRT_LIB=build_variants/libmyrt_pos.so $G" \
 "g_new2|200|$G" \
 "g_pos2|200|MYRT_LIB=build_variants/libmyrt_pos.so $G" \
 "c3g_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03r_c3g_trace -- python3 bench.py --config c3g --steps 10 --warmup 2 --in-flight 1 --no-cpu-baseline --no-side-paths"
for f in gpurun_out/g_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"one_frame_ms": [0-9.]*' $f)"; done
