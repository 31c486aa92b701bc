#!/bin/bash
# Round-4 check: incremental / API / scan parity with the per-prefix
# expansion and the cross-tile scan prefetch, then c3 and c4q A/B, then the
# reference's published experiment workloads.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_incremental_gpu.py tests/test_api_gpu.py tests/test_kernels_gpu.py \
  > gpurun_out/t_r04c.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r04c.log; exit 1; }
tail -1 gpurun_out/t_r04c.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_configs_gpu.py -k "c4 or c3" > gpurun_out/t_r04c_cfg.log 2>&1 || { echo "cfg rc=$?"; tail -30 gpurun_out/t_r04c_cfg.log; exit 1; }
tail -1 gpurun_out/t_r04c_cfg.log
timeout -k 10 120 python -u tools/bench_configs.py --only c3 > gpurun_out/c3_r04c_fused.jsonl 2>&1 || exit 1
DPF_AMD_PREFIX_EXPAND=0 timeout -k 10 120 python -u tools/bench_configs.py --only c3 > gpurun_out/c3_r04c_gather.jsonl 2>&1 || exit 1
tail -1 gpurun_out/c3_r04c_fused.jsonl; tail -1 gpurun_out/c3_r04c_gather.jsonl
bash tools/ab_c4q.sh 16,32,64,100 main noxt main noxt || exit 1
timeout -k 10 500 python -u bench.py --experiments --steps 3 > gpurun_out/experiments_r04c.jsonl 2> gpurun_out/experiments_r04c.err || { echo "experiments rc=$?"; tail -5 gpurun_out/experiments_r04c.err; exit 1; }
tail -1 gpurun_out/experiments_r04c.jsonl
# quad-lane walk A/B: 64 C++ EvaluateAt<uint128> calls of 16,384 points (c2)
for v in main quad0 rkm main quad0 rkm; do
  if [ "$v" = main ]; then LP=; else LP=$PWD/distributed_point_functions_amd/_native/var_$v; fi
  LD_LIBRARY_PATH=$LP timeout -k 10 120 distributed_point_functions_amd/_native/cpp_api_bench 5 c2 \
    > gpurun_out/cpp_c2_$v.log 2>&1 || { echo "cpp c2 $v failed"; tail -3 gpurun_out/cpp_c2_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/cpp_c2_$v.log)"
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_cpp_api.py \
  tests/test_multidevice_gpu.py > gpurun_out/t_r04c_cpp.log 2>&1 || { echo "cpp tests rc=$?"; tail -20 gpurun_out/t_r04c_cpp.log; exit 1; }
tail -1 gpurun_out/t_r04c_cpp.log
