B="python -u bench.py --config c5 --steps 400 --warmup 20 --no-cpu-baseline --no-side-paths"
G="python -u bench.py --config c3g --steps 20 --warmup 3 --no-cpu-baseline --no-side-paths"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
tools/gpu_session.sh \
 "lt|400|$T tests/test_gpu_features.py -k 'area or dielectric' tests/test_golden_frames.py tests/test_gpu_async.py" \
 "g_l1|200|$G" \
 "g_l0|200|MYRT_LEVELS=0 $G" \
 "g_f1|200|MYRT_FULL_FLIGHTS=1 $G" \
 "qt|300|$T tests/test_gpu_features.py tests/test_gpu_async.py -k 'queue or pipelined_mirror'" \
 "b_q0|200|$B" \
 "b_q1|200|MYRT_QUEUE=1 $B" \
 "b_q1_l0|200|MYRT_QUEUE=1 MYRT_QUEUE_LEVELS=0 $B" \
 "b_qp6|200|MYRT_QUEUE=1 MYRT_LIB=build_variants/libmyrt_qp6.so $B" \
 "b_qb6|200|MYRT_QUEUE=1 MYRT_LIB=build_variants/libmyrt_qb6.so $B" \
 "b_qpb6|200|MYRT_QUEUE=1 MYRT_LIB=build_variants/libmyrt_qpb6.so $B"
for f in gpurun_out/b_*.log gpurun_out/g_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
