#!/bin/bash
# Host-side A/Bs: EvaluateAt outputs written by the kernel into pinned host
# memory (DPF_AMD_HOST_OUT_KB) and a bounded spin of the host worker pool
# (DPF_AMD_POOL_SPIN_US).  Parity of both modes first (EvaluateAt /
# incremental / concurrency tests), then c2 (64 x C++ EvaluateAt) and c3
# (16 levels of EvaluateNext, HBM out) alternated.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 280 --timeout-method thread"
DPF_AMD_HOST_OUT_KB=4096 timeout -k 10 300 $T tests/test_configs_gpu.py tests/test_api_gpu.py \
  tests/test_incremental_gpu.py -k "c2 or evaluate_at or EvaluateAt" > gpurun_out/t_r04i_hostout.log 2>&1 \
  || { echo "hostout parity rc=$?"; tail -20 gpurun_out/t_r04i_hostout.log; exit 1; }
echo "hostout parity: $(tail -n 1 gpurun_out/t_r04i_hostout.log)"
for sp in 0 200; do
  DPF_AMD_POOL_SPIN_US=$sp timeout -k 10 400 $T tests/test_incremental_gpu.py tests/test_concurrency_gpu.py \
    > gpurun_out/t_r04i_spin$sp.log 2>&1 || { echo "spin=$sp parity rc=$?"; tail -20 gpurun_out/t_r04i_spin$sp.log; exit 1; }
  echo "spin=$sp parity: $(tail -n 1 gpurun_out/t_r04i_spin$sp.log)"
done
B=distributed_point_functions_amd/_native/cpp_api_bench
for ho in 0 4096 0 4096; do
  DPF_AMD_HOST_OUT_KB=$ho timeout -k 10 120 $B 5 c2 > gpurun_out/cpp_c2_ho${ho}_r04i.log 2>&1 || { echo "c2 ho=$ho failed"; exit 1; }
  echo "hostout=$ho $(tail -n 1 gpurun_out/cpp_c2_ho${ho}_r04i.log | cut -c1-160)"
done
for sp in 0 200 0 200; do
  DPF_AMD_POOL_SPIN_US=$sp timeout -k 10 150 python -u tools/bench_configs.py --only c3 > gpurun_out/c3_spin${sp}_r04i.jsonl 2>&1 \
    || { echo "c3 spin=$sp failed"; tail -3 gpurun_out/c3_spin${sp}_r04i.jsonl; exit 1; }
  echo "spin=$sp $(tail -n 1 gpurun_out/c3_spin${sp}_r04i.jsonl | cut -c1-220)"
done
DPF_AMD_POOL_SPIN_US=200 DPF_AMD_TRACE_HOST=1 timeout -k 10 100 $B 1 c3 > gpurun_out/cpp_c3_trace_spin200_r04i.log 2>&1 || exit 1
DPF_AMD_TRACE_HOST=1 timeout -k 10 100 $B 1 c3 > gpurun_out/cpp_c3_trace_spin0_r04i.log 2>&1 || exit 1
