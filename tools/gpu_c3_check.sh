#!/bin/bash
# c3 incremental path after a change: context / incremental parity tests, the
# Python device-output bench of c3 and the C++ API c3 with host phase times.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "incremental or c3 or context or partial or prefix or heavy or evaluate_next or golden or concurren" > gpurun_out/t_c3_$TAG.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_c3_$TAG.log; exit 1; }
tail -1 gpurun_out/t_c3_$TAG.log
timeout -k 10 300 python -u tools/bench_configs.py --only c3 > gpurun_out/cfg_c3_$TAG.log 2>&1 || { echo "cfg rc=$?"; tail -5 gpurun_out/cfg_c3_$TAG.log; exit 1; }
tail -1 gpurun_out/cfg_c3_$TAG.log | cut -c1-900
DPF_AMD_TRACE_HOST=1 timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 3 c3 > gpurun_out/cpp_c3_$TAG.log 2> gpurun_out/cpp_c3_trace_$TAG.log || { echo "bench rc=$?"; tail -5 gpurun_out/cpp_c3_trace_$TAG.log; exit 1; }
cat gpurun_out/cpp_c3_$TAG.log
