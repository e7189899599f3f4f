T=r03w
bash tools/gpu_session.sh \
 "${T}_c3i_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3i_trace -- python3 bench.py --config c3i --steps 20 --warmup 3 --in-flight 1 --no-cpu-baseline --no-side-paths" \
 "${T}_c3d_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3d_trace -- python3 bench.py --config c3d --steps 10 --warmup 2 --in-flight 1 --no-cpu-baseline --no-side-paths" \
 "${T}_c3g_pmc|300|timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAIT_ANY --output-format csv -d gpurun_out/${T}_c3g_pmc -- python3 bench.py --config c3g --steps 5 --warmup 1 --in-flight 1 --no-cpu-baseline --no-side-paths"
