#!/usr/bin/env bash
# Profiling session for the bench command (run on the GPU box via gpurun).
# usage: tools/prof_session.sh TAG [extra bench args...]
#   -> gpurun_out/TAG_*/ (rocprofv3 output) and gpurun_out/TAG_roofline.json (tools/pmc_roofline.py)
set -u
tag="$1"; shift
B="python3 bench.py --steps 20 --warmup 3 --in-flight 1 --no-cpu-baseline --no-side-paths $*"
# the frame's render kernel: <COUNT, BOUNCE, WALK (1 = identity, 2 = transformed), QUEUE>; C5 (mirror
# scene, render option queue = 1) is a frame chain: the queued primary pass, then per level
# k_bounce, the sparse last levels in one k_bounce_tail, then k_queue_done (tools/pmc_roofline.py sums
# it per frame)
KX=""
case " $* " in
  *" --config c5 "*) K="${KERNEL:-render_kernel<false, false, 1, true>}"
                     KX="--kernel 'k_bounce<1>' --kernel 'k_bounce_tail<1>' --kernel k_queue_done" ;;
  *" --config c3i "*) K="${KERNEL:-render_kernel<false, false, 3, false>}" ;;
  # full trace() frames (C3g / C3d: level passes; C3r: depth-first k_events): the frame chain
  *" --config c3g "*|*" --config c3d "*) K="${KERNEL:-k_level<1>}"
      KX="--kernel 'k_level_c<1>' --kernel k_ccount --kernel k_clist --kernel k_jofs --kernel k_jscan --kernel 'k_shade_c<1>' --kernel 'render_full<false, false, 1>'" ;;
  *" --config c3r "*) K="${KERNEL:-k_events<false, 1>}"
      KX="--kernel k_jscan --kernel k_ccount --kernel k_clist --kernel 'k_shade_c<1>' --kernel 'render_full<false, false, 1>'" ;;
  *) K="${KERNEL:-render_kernel<false, false, 1, false>}" ;;
esac
steps=(
  "${tag}_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_trace -- $B"
  "${tag}_fetch|300|timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_fetch -- $B"
  "${tag}_write|300|timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_write -- $B"
  "${tag}_td|300|timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TD_TD_BUSY_sum --output-format csv -d gpurun_out/${tag}_td -- $B"
  "${tag}_valu|300|timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/${tag}_valu -- $B"
  "${tag}_sq|300|timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS --output-format csv -d gpurun_out/${tag}_sq -- $B"
  "${tag}_mix|300|timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d gpurun_out/${tag}_mix -- $B"
  "${tag}_ta|300|timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum --output-format csv -d gpurun_out/${tag}_ta -- $B"
  "${tag}_roofline|60|python3 tools/pmc_roofline.py --kernel '$K' $KX --trace gpurun_out/${tag}_trace --fetch gpurun_out/${tag}_fetch --write gpurun_out/${tag}_write --td gpurun_out/${tag}_td --valu gpurun_out/${tag}_valu --sq gpurun_out/${tag}_sq --lib myraytracer_amd/libmyrt.so -o gpurun_out/${tag}_roofline.json"
)
bash "$(dirname "$0")/gpu_session.sh" "${steps[@]}"
