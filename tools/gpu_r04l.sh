#!/bin/bash
# Host path of EvaluateUntil: stored-order check fused with the merge join,
# context rewrite in place over the host pool.  Incremental / API /
# concurrency / c3 parity, then c3 device-out A/B against the previous build
# (var_old) alternated, and a host-phase trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_api_gpu.py \
  tests/test_incremental_gpu.py tests/test_concurrency_gpu.py tests/test_wire_gpu.py tests/test_configs_gpu.py \
  -k "not c4 and not c2" > gpurun_out/t_r04l.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_r04l.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/t_r04l.log)"
for v in main old main old main old; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 150 python -u tools/bench_configs.py --only c3 > gpurun_out/c3_r04l_$v.jsonl 2>&1 || exit 1
  tail -n 1 gpurun_out/c3_r04l_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v c3 device_out_ms_total %.2f host_out_ms_total %.1f' % (d['device_out_ms_total'], d['host_out_ms_total']))"
done
unset DPF_AMD_LIB
DPF_AMD_TRACE_HOST=1 timeout -k 10 100 distributed_point_functions_amd/_native/cpp_api_bench 1 c3 \
  > gpurun_out/cpp_c3_trace_r04l.log 2>&1 || exit 1
