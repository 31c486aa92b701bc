#!/bin/bash
# A/B of the c3 level's correction-word upload on one box: the GPU suite's
# hierarchical / incremental tests, then tools/bench_configs.py c3 alternated
# between the default (correction words host-written into fine-grained VRAM)
# and DPF_AMD_HOST_WRITE=0 (a copy kernel per level).
# Usage: bash tools/ab_c3_place.sh <tag>
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/ab_c3_place_${TAG}.log
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_c3_tests_${TAG}.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/ab_c3_tests_${TAG}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_c3_tests_${TAG}.log)" | tee $OUT
for round in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then E="DPF_AMD_HOST_WRITE=0"; else E="DPF_AMD_HOST_WRITE=1"; fi
    echo "== $v round=$round" >> $OUT
    env $E timeout -k 10 200 python -u tools/bench_configs.py --only c3 --no-ab 2>&1 | grep -v amdgpu.ids >> $OUT \
      || { echo "c3 rc=$?"; tail -20 $OUT; exit 1; }
  done
done
cut -c1-400 $OUT
