G="python -u bench.py --config c3g --steps 20 --warmup 3 --no-cpu-baseline --no-side-paths"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
tools/gpu_session.sh \
 "suite|600|$T tests -m gpu" \
 "g_f2|200|MYRT_FULL_FLIGHTS=2 $G" \
 "g_f8|200|MYRT_FULL_FLIGHTS=8 $G" \
 "g_f16|200|MYRT_FULL_FLIGHTS=16 $G" \
 "g_f4|200|$G" \
 "c3g_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03q_c3g_trace -- python3 bench.py --config c3g --steps 10 --warmup 2 --in-flight 1 --no-cpu-baseline --no-side-paths"
for f in gpurun_out/g_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
