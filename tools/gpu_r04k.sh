#!/bin/bash
# Range check fused into the de-duplication pass: the range-error test and the
# incremental / API suites, then a host-phase trace of the C++ c3 path and
# the c3 device-out bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_api_gpu.py \
  tests/test_incremental_gpu.py tests/test_configs_gpu.py -k "not c4 and not c2" > gpurun_out/t_r04k.log 2>&1 \
  || { echo "tests rc=$?"; tail -20 gpurun_out/t_r04k.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/t_r04k.log)"
DPF_AMD_TRACE_HOST=1 timeout -k 10 100 distributed_point_functions_amd/_native/cpp_api_bench 1 c3 \
  > gpurun_out/cpp_c3_trace_r04k.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python -u tools/bench_configs.py --only c3 > gpurun_out/c3_r04k_$i.jsonl 2>&1 || exit 1
  tail -n 1 gpurun_out/c3_r04k_$i.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 device_out_ms_total', d['device_out_ms_total'])"
done
