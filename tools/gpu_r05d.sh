#!/bin/bash
# Round 5: per-call EvaluateAt overhead A/B — spin-then-block stream wait
# (DPF_AMD_WAIT_SPIN_US) and the pooled copy out of pinned memory
# (DPF_AMD_COPY_GRAIN_KB), alternated, 64 C++ EvaluateAt calls each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B=distributed_point_functions_amd/_native/cpp_api_bench
L=gpurun_out/c2_wait_ab_r05d.log
: > $L
for rep in 1 2; do
  for v in "0 0" "200 0" "0 64" "200 64" "1000 64" "200 32"; do
    set -- $v
    echo -n "spin=$1 grain=$2 " >> $L
    DPF_AMD_WAIT_SPIN_US=$1 DPF_AMD_COPY_GRAIN_KB=$2 timeout -k 10 60 $B 9 c2 >> $L 2>&1 || { echo "rc=$?"; tail $L; exit 1; }
  done
done
cat $L
DPF_AMD_TRACE_HOST=1 timeout -k 10 60 $B 1 c2 > gpurun_out/cpp_c2_trace_r05d.log 2>&1 && grep EvaluateAt gpurun_out/cpp_c2_trace_r05d.log | tail -7
