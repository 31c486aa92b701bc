#!/bin/bash
# Main build (P = 4 scan lanes mapped onto the ds_read_b128 lane groups; quad
# rounds with the DPP moves after the lookups): parity on the scan, c4 and
# quad-walk tests, then the Q = 16 / 24 scan A/B against the linear lane map
# (var_p4lin), the 64 x EvaluateAt A/B against the previous quad round
# (var_pd0), and a PMC profile of the Q = 16 scan.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "inner_product or scan or c4 or quad or c2 or points" \
  > gpurun_out/t_r04g_main.log 2>&1 || { echo "main parity rc=$?"; tail -20 gpurun_out/t_r04g_main.log; exit 1; }
echo "main parity: $(tail -1 gpurun_out/t_r04g_main.log)"
bash tools/ab_c4q.sh 16,24 main p4lin main p4lin || exit 1
for v in main pd0 main pd0; do
  if [ "$v" = main ]; then LP=; else LP=$PWD/distributed_point_functions_amd/_native/var_$v; fi
  LD_LIBRARY_PATH=$LP timeout -k 10 120 distributed_point_functions_amd/_native/cpp_api_bench 5 c2 \
    > gpurun_out/cpp_c2_r04g_$v.log 2>&1 || { echo "cpp c2 $v failed"; tail -3 gpurun_out/cpp_c2_r04g_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/cpp_c2_r04g_$v.log)"
done
ARGS="--only c4q --c4q-queries 16 --no-ab --reps 3" bash tools/profile_configs.sh r04q16g || exit 1
