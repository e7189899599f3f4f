G="python -u bench.py --config c3g --steps 30 --warmup 3 --no-cpu-baseline --no-side-paths"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
tools/gpu_session.sh \
 "lt|400|MYRT_TREE_PPW=2 $T tests/test_gpu_features.py tests/test_gpu_async.py tests/test_golden_frames.py -k 'area or dielectric or full_trace or glass'" \
 "g_p1|200|MYRT_TREE_PPW=1 $G" \
 "g_p2|200|MYRT_TREE_PPW=2 $G" \
 "g_p4|200|MYRT_TREE_PPW=4 $G" \
 "g_p8|200|MYRT_TREE_PPW=8 $G" \
 "g_p16|200|MYRT_TREE_PPW=16 $G" \
 "g_p1b|200|MYRT_TREE_PPW=1 $G" \
 "g_p4b|200|MYRT_TREE_PPW=4 $G"
for f in gpurun_out/g_p*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"one_frame_ms": [0-9.]*' $f)"; done
