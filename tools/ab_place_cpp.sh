#!/bin/bash
# A/B of the host-written inputs (EvaluateUntil's root + correction words,
# EvaluateAndApply's level block, c3's correction words) on one box: the GPU
# suite, then the C++ API bench and the c3 config alternated between the
# default and DPF_AMD_HOST_WRITE=0 (copy kernels).
# Usage: bash tools/ab_place_cpp.sh <tag>
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/ab_place_cpp_${TAG}.log
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_place_tests_${TAG}.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/ab_place_tests_${TAG}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_place_tests_${TAG}.log)" | tee $OUT
for round in 1 2; do
  for v in new old; do
    if [ $v = old ]; then E="DPF_AMD_HOST_WRITE=0"; else E="DPF_AMD_HOST_WRITE=1"; fi
    echo "== $v round=$round" >> $OUT
    env $E timeout -k 10 200 ./distributed_point_functions_amd/_native/cpp_api_bench 6 2>&1 | grep -v amdgpu.ids | cut -c1-200 >> $OUT \
      || { echo "cpp rc=$?"; tail -20 $OUT; exit 1; }
    env $E timeout -k 10 200 python -u tools/bench_configs.py --only c3 --no-ab 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c3 device_out_ms_total', round(d['device_out_ms_total'],3), d['device_out_ms_per_level'][3:8])" >> $OUT \
      || { echo "c3 rc=$?"; tail -20 $OUT; exit 1; }
  done
done
cat $OUT
