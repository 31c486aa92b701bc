#!/bin/bash
# A/B of the latency-bound launches across library variants (GPU box): the
# parity tests of the quad walk and the cooperative expansion on the main
# build, then per variant, alternated: c1's kernel (bench_configs c1), 64 C++
# EvaluateAt calls (cpp_api_bench c2), one rank's c4/8 request at Q = 1
# (pir_hr_probe --log-n 23).  Usage: bash tools/ab_latency.sh <tag> <rounds> main var1 ...
set -o pipefail
TAG=${1:?tag}
ROUNDS=${2:?rounds}
shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
LOG=gpurun_out/ab_latency_${TAG}.log
N=distributed_point_functions_amd/_native
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py -x -q \
  --timeout 300 --timeout-method thread \
  -k "evaluate_points or cooperative or leaf_ranges or roots_stage or automatic" \
  > gpurun_out/ab_latency_tests_${TAG}.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/ab_latency_tests_${TAG}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_latency_tests_${TAG}.log)" | tee $LOG
for v in "$@"; do
  if [ "$v" != main ]; then cp $N/cpp_api_bench $N/var_$v/; fi
done
for i in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ "$v" = main ]; then export DPF_AMD_LIB=; B=$N/cpp_api_bench; else
      export DPF_AMD_LIB=$PWD/$N/var_$v/libdpf_amd.so; B=$N/var_$v/cpp_api_bench; fi
    timeout -k 10 120 python -u tools/bench_configs.py --only c1 --reps 40 \
      > gpurun_out/ab_lat_c1.log 2>&1 || { echo "c1 $v failed"; tail -5 gpurun_out/ab_lat_c1.log; exit 1; }
    c1=$(tail -1 gpurun_out/ab_lat_c1.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_ms']*1e3, 1), d['correct'])")
    timeout -k 10 120 $B 6 c2 > gpurun_out/ab_lat_c2.log 2>&1 \
      || { echo "c2 $v failed"; tail -5 gpurun_out/ab_lat_c2.log; exit 1; }
    c2=$(grep '"config": "c2"' gpurun_out/ab_lat_c2.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['best_ms'], d['correct'])")
    timeout -k 10 120 python -u tools/pir_hr_probe.py --log-n 23 --queries 1 --reps 20 \
      > gpurun_out/ab_lat_hr.log 2>&1 || { echo "hr $v failed"; tail -5 gpurun_out/ab_lat_hr.log; exit 1; }
    hr=$(tail -1 gpurun_out/ab_lat_hr.log)
    echo "$v c1_kernel_us=$c1 | c2_64_calls_ms=$c2 | $hr" | tee -a $LOG
  done
done
