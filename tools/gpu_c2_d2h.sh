#!/bin/bash
# C++ EvaluateAt loop (c2) with the D2H staging threshold at 1 MiB / 64 KiB
# / 16 KiB, per-call host phases with DPF_AMD_TRACE_HOST (gpurun).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "evaluate_at or point or apply or incremental" > gpurun_out/t_c2d.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_c2d.log; exit 1; }
tail -1 gpurun_out/t_c2d.log
for kb in 1024 64 16; do
  DPF_AMD_D2H_DIRECT_KB=$kb timeout -k 10 200 distributed_point_functions_amd/_native/cpp_api_bench 5 c2 > gpurun_out/c2d_$kb.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  echo "direct<=${kb}KiB: $(cat gpurun_out/c2d_$kb.log)"
done
DPF_AMD_TRACE_HOST=1 timeout -k 10 200 distributed_point_functions_amd/_native/cpp_api_bench 2 c2 > /dev/null 2> gpurun_out/c2d_trace.log || exit 1
grep "EvaluateAt/" gpurun_out/c2d_trace.log | tail -5
