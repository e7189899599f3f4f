#!/usr/bin/env bash
# The round's final measurement session (run on the GPU box via gpurun): PMC + kernel-trace
# profiles of C3/C5 (tools/prof_session.sh), the bench loop's kernel overlap
# (tools/overlap_session.sh), a one-pass VALU PMC of the full trace() frames (C3g, C3r), smoke,
# bench lines of every config and the GPU suite.
# usage: gpurun -- 'bash tools/final_session.sh TAG [1|2]'  ->  gpurun_out/TAG_*
#   part 1 = the PMC / kernel-trace / overlap profiles, part 2 = smoke, bench lines, full-trace
#   profiles and the GPU suite, part 3 = the PMC profiles of C3i / C3g / C3r / C3d / C2 (each fits
#   one gpurun call); no part = 1 and 2
set -u
T="${1:-r04z}"
PART="${2:-all}"
G="python3 bench.py --steps 10 --warmup 2 --in-flight 1 --no-cpu-baseline --no-side-paths"
VALU="GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
if [ "$PART" = 1 ] || [ "$PART" = all ]; then
bash tools/prof_session.sh ${T}_c3 || exit $?
bash tools/prof_session.sh ${T}_c5 --config c5 || exit $?
bash tools/overlap_session.sh ${T}_c3 c3 300 || exit $?
bash tools/overlap_session.sh ${T}_c5 c5 100 || exit $?
fi
if [ "$PART" = 3 ]; then      # part 3: the roofline profiles of the other configs (bench reads roofline_<config>.json)
for c in c3i c3g c3r c3d c2; do bash tools/prof_session.sh ${T}_$c --config $c || exit $?; done
exit 0
fi
[ "$PART" = 1 ] && exit 0
[ "$PART" = 3 ] && exit 0
bash tools/gpu_session.sh \
 "${T}_smoke|300|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "${T}_bc3|300|python3 bench.py > gpurun_out/${T}_bench_c3.json" \
 "${T}_bc5|300|python3 bench.py --config c5 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_bench_c5.json" \
 "${T}_bc3i|300|python3 bench.py --config c3i --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_bench_c3i.json" \
 "${T}_bc3g|300|python3 bench.py --config c3g --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench_c3g.json" \
 "${T}_bc3r|300|python3 bench.py --config c3r --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench_c3r.json" \
 "${T}_bc3d|300|python3 bench.py --config c3d --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench_c3d.json" \
 "${T}_bc2|300|python3 bench.py --config c2 --steps 2000 --warmup 50 > gpurun_out/${T}_bench_c2.json" \
 "${T}_bc3k|300|python3 bench.py --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/${T}_bench_c3_2000.json" \
 "${T}_c3g_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3g_trace -- $G --config c3g" \
 "${T}_c3r_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3r_trace -- $G --config c3r" \
 "${T}_c3g_valu|300|timeout -s KILL 240 rocprofv3 --pmc $VALU --output-format csv -d gpurun_out/${T}_c3g_valu -- $G --config c3g" \
 "${T}_c3r_valu|300|timeout -s KILL 240 rocprofv3 --pmc $VALU --output-format csv -d gpurun_out/${T}_c3r_valu -- $G --config c3r" || exit $?
bash tools/gpu_session.sh \
 "${T}_suite|700|python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu"
