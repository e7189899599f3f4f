D="python -u bench.py --config c3d --steps 30 --warmup 3 --no-cpu-baseline --no-side-paths"
T="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
tools/gpu_session.sh \
 "dt|700|$T tests/test_gpu_features.py tests/test_gpu_frames.py -k 'dielectric or area or general_path'" \
 "d_l1|200|$D" \
 "d_l0|200|MYRT_LEVELS=0 $D" \
 "d_l1b|200|$D" \
 "d_l0b|200|MYRT_LEVELS=0 $D"
for f in gpurun_out/d_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"one_frame_ms": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f)"; done
