#!/bin/bash
# Round 5: where the per-call time goes in the C++ API configs — c2 (64 x
# EvaluateAt), c1 (EvaluateNext 2^20) and c3 (16 incremental levels): host
# phase times (DPF_AMD_TRACE_HOST) and a kernel trace of each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B=distributed_point_functions_amd/_native/cpp_api_bench
timeout -k 10 120 $B 5 c1,c2,c3 > gpurun_out/cpp_r05c.log 2>&1 || { echo "bench rc=$?"; tail gpurun_out/cpp_r05c.log; exit 1; }
cat gpurun_out/cpp_r05c.log
DPF_AMD_TRACE_HOST=1 timeout -k 10 120 $B 1 c2 > gpurun_out/cpp_c2_trace_r05c.log 2>&1 || { echo "c2 trace rc=$?"; exit 1; }
DPF_AMD_TRACE_HOST=1 timeout -k 10 120 $B 1 c3 > gpurun_out/cpp_c3_trace_r05c.log 2>&1 || { echo "c3 trace rc=$?"; exit 1; }
for c in c1 c2 c3; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ktrace_${c}_r05c -o tr \
    --output-format csv -- $B 1 $c > gpurun_out/ktrace_${c}_r05c.log 2>&1 || { echo "ktrace $c rc=$?"; exit 1; }
done
echo done
