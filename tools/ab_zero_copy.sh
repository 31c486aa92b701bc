#!/bin/bash
# A/B of one EvaluateAt call's point input read in place from the pinned
# slot (zero-copy, default) against the copy kernel (DPF_AMD_ZERO_COPY=0):
# the API / C-ABI / C++ tests under the default, then 64 C++ EvaluateAt calls
# (cpp_api_bench c2) alternated.  Usage: bash tools/ab_zero_copy.sh <tag> <rounds>
set -o pipefail
TAG=${1:?tag}
ROUNDS=${2:?rounds}
export TMPDIR=/tmp
mkdir -p gpurun_out
LOG=gpurun_out/ab_zero_copy_${TAG}.log
B=distributed_point_functions_amd/_native/cpp_api_bench
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "evaluate_at or EvaluateAt or golden or incremental or cpp or points or experiments" \
  > gpurun_out/ab_zc_tests_${TAG}.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/ab_zc_tests_${TAG}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_zc_tests_${TAG}.log)" | tee $LOG
for i in $(seq 1 $ROUNDS); do
  for z in 1 0; do
    DPF_AMD_ZERO_COPY=$z timeout -k 10 120 $B 6 c2 > gpurun_out/ab_zc_c2.log 2>&1 \
      || { echo "c2 z=$z failed"; tail -5 gpurun_out/ab_zc_c2.log; exit 1; }
    echo "zero_copy=$z $(grep '"c2"' gpurun_out/ab_zc_c2.log)" | tee -a $LOG
  done
done
