#!/bin/bash
# Quad-lane walk A/B: lookups on the lane's own bytes with the DPP moves after
# them (pd1: separate moves, pd2: moves folded into VOP2 XORs) against the
# main build — parity of the forced quad walk and the c2 shapes first, then 64
# C++ EvaluateAt<uint128> calls of 16,384 points, alternated.  Then a PMC
# profile of the Q = 16 many-query scan.
set -o pipefail
mkdir -p gpurun_out
var() { echo $PWD/distributed_point_functions_amd/_native/var_$1; }
for v in pd1 pd2; do
  DPF_AMD_LIB=$(var $v)/libdpf_amd.so timeout -k 10 300 python -u -m pytest -x -v --timeout 280 \
    --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py -k "quad or c2 or points" \
    > gpurun_out/t_r04f_$v.log 2>&1 || { echo "$v parity rc=$?"; tail -20 gpurun_out/t_r04f_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/t_r04f_$v.log)"
done
for v in main pd1 pd2 main pd1 pd2; do
  if [ "$v" = main ]; then LP=; else LP=$(var $v); fi
  LD_LIBRARY_PATH=$LP timeout -k 10 120 distributed_point_functions_amd/_native/cpp_api_bench 5 c2 \
    > gpurun_out/cpp_c2_r04f_$v.log 2>&1 || { echo "cpp c2 $v failed"; tail -3 gpurun_out/cpp_c2_r04f_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/cpp_c2_r04f_$v.log)"
done
ARGS="--only c4q --c4q-queries 16 --no-ab --reps 3" bash tools/profile_configs.sh r04q16 || exit 1
