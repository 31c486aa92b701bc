#!/bin/bash
# A/B of Four-Russians scan variants at 33-100 queries (library variants from
# tools/build_variants.py): the scan / c4 / API PIR tests on the default,
# then c4 scans at Q = 33 / 40 / 48 / 64 / 100 per variant, alternated.
# Usage: bash tools/ab_scan_pair.sh <tag> <rounds> main <variant>...
set -o pipefail
TAG=${1:?tag}
ROUNDS=${2:?rounds}
shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
LOG=gpurun_out/ab_scan_pair_${TAG}.log
N=distributed_point_functions_amd/_native
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_api_gpu.py tests/test_configs_gpu.py -x -q \
  --timeout 300 --timeout-method thread -k "inner_product or scan or pir or c4" \
  > gpurun_out/ab_sp_tests_${TAG}.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/ab_sp_tests_${TAG}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_sp_tests_${TAG}.log)" | tee $LOG
for i in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ $v = main ]; then export DPF_AMD_LIB=; else export DPF_AMD_LIB=$PWD/$N/var_$v/libdpf_amd.so; fi
    timeout -k 10 300 python -u tools/bench_configs.py --only c4q --c4q-queries 40,64,80,100,112 --no-ab \
      > gpurun_out/ab_sp.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_sp.log; exit 1; }
    tail -1 gpurun_out/ab_sp.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', {k: round(v,3) for k,v in d.items() if k.endswith('_ms')})" | tee -a $LOG
  done
done
