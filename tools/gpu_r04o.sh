#!/bin/bash
# Table fill by scalar row chunks (main) against the per-word vector loads
# (var_fill0): the full -m gpu suite on main, then c1 and 64 x EvaluateAt
# alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r04o.log 2>&1 || { echo "gpu tests rc=$?"; tail -20 gpurun_out/gpu_tests_r04o.log; exit 1; }
tail -n 1 gpurun_out/gpu_tests_r04o.log
B=distributed_point_functions_amd/_native/cpp_api_bench
for v in main fill0 main fill0 main fill0; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; LP=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so
    LP=$PWD/distributed_point_functions_amd/_native/var_$v; fi
  timeout -k 10 150 python -u tools/bench_configs.py --only c1 > gpurun_out/c1_r04o_$v.jsonl 2>&1 || exit 1
  LD_LIBRARY_PATH=$LP timeout -k 10 120 $B 5 c2 > gpurun_out/cpp_c2_r04o_$v.log 2>&1 || exit 1
  echo "$v c1 $(tail -n 1 gpurun_out/c1_r04o_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms %.4f' % d['kernel_ms'])") c2 $(tail -n 1 gpurun_out/cpp_c2_r04o_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('best_ms %.3f' % d['best_ms'])")"
done
