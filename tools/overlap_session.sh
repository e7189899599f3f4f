#!/usr/bin/env bash
# Kernel concurrency of bench.py's own pipelined loop (16 renders in flight, 32 HW queues):
# rocprofv3 --kernel-trace over the bench, then tools/overlap_summary.py on the timed frames,
# plus a same-build bench run without the profiler for its ms_per_step.
# usage: tools/overlap_session.sh TAG CONFIG STEPS [WARMUP]
#   -> gpurun_out/TAG_pipe/ (trace), TAG_pipe_bench.json, TAG_bench.json, TAG_overlap.json
set -u
tag="$1"; cfg="$2"; steps="$3"; warm="${4:-50}"
KX=""
case "$cfg" in
  # C5 (render option queue = 1): the queued primary pass + the per-level launches of its frame
  c5) K="${KERNEL:-render_kernel<false, false, 1, true>}"
      KX="--extra-kernel 'k_bounce<1>' --extra-kernel k_queue_done" ;;
  *)  K="${KERNEL:-render_kernel<false, false, 1, false>}" ;;
esac
B="python3 bench.py --config $cfg --steps $steps --warmup $warm --no-cpu-baseline --no-side-paths"
s=(
  "${tag}_bench|400|$B > gpurun_out/${tag}_bench.json"
  "${tag}_pipe|400|rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_pipe -- $B > gpurun_out/${tag}_pipe_bench.json"
  "${tag}_overlap|120|python3 tools/overlap_summary.py --trace gpurun_out/${tag}_pipe --kernel '$K' $KX --skip $((warm + 16)) --frames $steps --bench gpurun_out/${tag}_pipe_bench.json --lib myraytracer_amd/libmyrt.so -o gpurun_out/${tag}_overlap.json"
)
bash "$(dirname "$0")/gpu_session.sh" "${s[@]}"
