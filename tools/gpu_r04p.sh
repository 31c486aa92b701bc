#!/bin/bash
# KExpandCoop with four tables and the four-table quad round in its walk when
# the launch has at most one block per CU (main) against two tables
# (var_coopt2, the uint64 TU): expansion parity (all forced kernel shapes +
# configs), then c1 and the C++ HandleRequest Q = 1 alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py \
  tests/test_kernels_gpu.py tests/test_configs_gpu.py -k "not c5_full_domain_every and not eight_rank" \
  > gpurun_out/t_r04p.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_r04p.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/t_r04p.log)"
for v in main coopt2 main coopt2 main coopt2; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 150 python -u tools/bench_configs.py --only c1 > gpurun_out/c1_r04p_$v.jsonl 2>&1 || exit 1
  echo "$v c1 $(tail -n 1 gpurun_out/c1_r04p_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms %.4f api_ms %.3f' % (d['kernel_ms'], d['api_ms']))")"
done
