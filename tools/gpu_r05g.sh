#!/bin/bash
# Round 5: c3 after the pooled prefix upload and the size query without the
# range check; EvaluateAt (c2) unchanged check; the incremental tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_incremental_gpu.py tests/test_api_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/t_r05g.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r05g.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_r05g.log)"
for m in dev host dev; do
  if [ $m = host ]; then export DPF_AMD_HOST_INCREMENTAL=1; else unset DPF_AMD_HOST_INCREMENTAL; fi
  timeout -k 10 200 python -u tools/bench_configs.py --only c3 --reps 8 > gpurun_out/c3_${m}_r05g.log 2>&1 \
    || { echo "c3 $m rc=$?"; tail gpurun_out/c3_${m}_r05g.log; exit 1; }
  echo "$m: $(tail -1 gpurun_out/c3_${m}_r05g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["device_out_ms_total"], d["device_out_ms_per_level"][2:6], d["host_out_ms_total"], d["correct"])')"
done
unset DPF_AMD_HOST_INCREMENTAL
B=distributed_point_functions_amd/_native/cpp_api_bench
timeout -k 10 120 $B 5 c2,c3 > gpurun_out/cpp_r05g.log 2>&1 && cat gpurun_out/cpp_r05g.log | cut -c1-300
DPF_AMD_TRACE_HOST=1 timeout -k 10 200 python -u tools/bench_configs.py --only c3 --reps 2 > gpurun_out/c3_trace_r05g.log 2>&1 || true
