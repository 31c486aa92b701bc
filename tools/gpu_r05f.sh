#!/bin/bash
# Round 5: EvaluateUntil's device-resident bookkeeping (de-duplication,
# stored-evaluation lookup and the context's list in HBM): the incremental,
# c3, API and sharding tests, then c3 timed device path vs host path.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_incremental_gpu.py tests/test_configs_gpu.py \
  tests/test_api_gpu.py tests/test_sharding_gpu.py tests/test_concurrency_gpu.py tests/test_cpp_api.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -k "incremental or c3 or ctx or evaluate_until or context or concurren or cpp or shard or device_bookkeeping" \
  > gpurun_out/t_r05f.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/t_r05f.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_r05f.log)"
for m in dev host dev host; do
  if [ $m = host ]; then export DPF_AMD_HOST_INCREMENTAL=1; else unset DPF_AMD_HOST_INCREMENTAL; fi
  timeout -k 10 200 python -u tools/bench_configs.py --only c3 --reps 8 > gpurun_out/c3_${m}_r05f.log 2>&1 \
    || { echo "c3 $m rc=$?"; tail gpurun_out/c3_${m}_r05f.log; exit 1; }
  echo "$m: $(tail -1 gpurun_out/c3_${m}_r05f.log | cut -c1-600)"
done
unset DPF_AMD_HOST_INCREMENTAL
DPF_AMD_TRACE_HOST=1 timeout -k 10 200 python -u tools/bench_configs.py --only c3 --reps 4 > gpurun_out/c3_trace_r05f.log 2>&1 || true
