B="python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline --no-side-paths"
tools/gpu_session.sh \
 "p_c3|300|python -u tools/probe_lib.py c3 build_variants/libmyrt_base.so build_variants/libmyrt_nsf.so" \
 "p_c5|300|python -u tools/probe_lib.py c5 build_variants/libmyrt_base.so build_variants/libmyrt_nsf.so" \
 "p_c3i|300|python -u tools/probe_lib.py c3i build_variants/libmyrt_base.so build_variants/libmyrt_nsf.so" \
 "b_base|200|MYRT_LIB=build_variants/libmyrt_base.so $B" \
 "b_nsf|200|MYRT_LIB=build_variants/libmyrt_nsf.so $B" \
 "b_base2|200|MYRT_LIB=build_variants/libmyrt_base.so $B" \
 "b_nsf2|200|MYRT_LIB=build_variants/libmyrt_nsf.so $B"
for f in gpurun_out/b_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
