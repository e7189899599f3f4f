#!/usr/bin/env bash
# Profiling session for the default bench command (run on the GPU box via gpurun).
# usage: tools/prof_session.sh TAG [extra bench args...]
set -u
tag="$1"; shift
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path $*"
exec_steps=(
  "${tag}_trace|400|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_trace -- $B"
  "${tag}_fetch|400|rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_fetch -- $B"
  "${tag}_write|400|rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_write -- $B"
  "${tag}_sq1|400|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_BRANCH --output-format csv -d gpurun_out/${tag}_sq1 -- $B"
  "${tag}_sq2|400|rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d gpurun_out/${tag}_sq2 -- $B"
  "${tag}_td|400|rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TD_TD_BUSY_sum SQ_THREAD_CYCLES_VALU --output-format csv -d gpurun_out/${tag}_td -- $B"
  "${tag}_valu|400|rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 --output-format csv -d gpurun_out/${tag}_valu -- $B"
  "${tag}_tc|400|rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/${tag}_tc -- $B"
)
bash "$(dirname "$0")/gpu_session.sh" "${exec_steps[@]}"
