#!/usr/bin/env bash
# A/B of near-root BLAS records staged in LDS (MYRT_LDS_TOP) with TD busy, C3 and C5.
# Built with a 12-entry LDS stack so 31 records (2 KB/wave) fit beside the pixel slots
# at 16 waves/CU.  usage (GPU box): bash tools/ab_ldstop.sh  -> gpurun_out/ldstop_*
set -u
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-side-paths"
steps=()
for cfg in c3 c5; do
  K='render_kernel<false, false, true>'; [ $cfg = c5 ] && K='render_kernel<false, true, true>'
  for top in 0 31; do
    t="ldstop_${cfg}_${top}"
    steps+=("${t}_trace|300|MYRT_LIB=build_variants/libmyrt_klds12.so MYRT_LDS_TOP=$top rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_trace -- $B --config $cfg")
    steps+=("${t}_td|300|MYRT_LIB=build_variants/libmyrt_klds12.so MYRT_LDS_TOP=$top timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TD_TD_BUSY_sum SQ_THREAD_CYCLES_VALU --output-format csv -d gpurun_out/${t}_td -- $B --config $cfg")
  done
done
bash "$(dirname "$0")/gpu_session.sh" "${steps[@]}"
