#!/bin/bash
# c3 bookkeeping in one kernel (DedupLookup: de-duplication + context lookup,
# decoupled look-back) against the previous library (var_old: three dedup
# kernels + a lookup kernel): the incremental / c3 tests on the new build,
# then c3 levels alternated.  Usage: bash tools/ab_c3_fused.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:?tag}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
OUT=gpurun_out/ab_${T}.log
: > $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_incremental_gpu.py tests/test_configs_gpu.py tests/test_api_gpu.py -k "incremental or c3 or context or evaluate_until or prefix or hierarch" > gpurun_out/t_${T}.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_${T}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_${T}.log)" | tee -a $OUT
for rep in 1 2 3; do
  for v in old main; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u tools/bench_configs.py --only c3 > gpurun_out/ab_${T}_c3_${v}.jsonl 2>&1 || { echo "c3 rc=$?"; tail gpurun_out/ab_${T}_c3_${v}.jsonl; exit 1; }
    echo "c3 $v $rep $(tail -1 gpurun_out/ab_${T}_c3_${v}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['device_out_ms_total'],3), d['device_out_ms_per_level'][2:10], round(d['host_out_ms_total'],1))")" | tee -a $OUT
  done
done
echo done
