#!/bin/bash
# Partial-evaluation lookup: stored-order check and merge join in one pool
# job (main) or two (var_unfused).  Parity of both on the incremental tests,
# then c3 device-out alternated.
set -o pipefail
mkdir -p gpurun_out
for v in main unfused; do
  if [ "$v" = main ]; then L=; else L=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  DPF_AMD_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
    tests/test_incremental_gpu.py tests/test_api_gpu.py -k "incremental or context or prefix" \
    > gpurun_out/t_r04m_$v.log 2>&1 || { echo "$v tests rc=$?"; tail -20 gpurun_out/t_r04m_$v.log; exit 1; }
  echo "$v tests: $(tail -n 1 gpurun_out/t_r04m_$v.log)"
done
for v in main unfused main unfused main unfused; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 150 python -u tools/bench_configs.py --only c3 > gpurun_out/c3_r04m_$v.jsonl 2>&1 || exit 1
  tail -n 1 gpurun_out/c3_r04m_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v c3 device_out_ms_total %.2f' % d['device_out_ms_total'])"
done
