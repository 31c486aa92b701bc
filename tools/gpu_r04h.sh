#!/bin/bash
# D2H completion wait A/B through the C++ API (c1 EvaluateNext, c2 64 x
# EvaluateAt, c4 HandleRequest): hipEventSynchronize (default) against
# polling (DPF_AMD_SPIN_WAIT=1), alternated; then one host-phase trace of c2
# per mode.
set -o pipefail
mkdir -p gpurun_out
B=distributed_point_functions_amd/_native/cpp_api_bench
for sp in 0 1 0 1; do
  DPF_AMD_SPIN_WAIT=$sp timeout -k 10 200 $B 5 c1,c2,c4 > gpurun_out/cpp_spin${sp}_r04h_$RANDOM.log 2>&1 \
    || { echo "spin=$sp failed"; exit 1; }
  echo "spin=$sp"; tail -n 8 $(ls -t gpurun_out/cpp_spin${sp}_r04h_*.log | head -n 1) | cut -c1-200
done
for sp in 0 1; do
  DPF_AMD_TRACE_HOST=1 DPF_AMD_SPIN_WAIT=$sp timeout -k 10 100 $B 1 c2 > gpurun_out/cpp_c2_trace_spin${sp}_r04h.log 2>&1 \
    || { echo "trace spin=$sp failed"; exit 1; }
done
