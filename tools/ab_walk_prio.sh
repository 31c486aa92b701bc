#!/bin/bash
# Progress-ordered wave priority in the lane-per-point walks (variant `wp`,
# DPF_WALK_PRIO=1) against the main build: the point / seed walk tests and
# c2 at full size on the variant, then c2's batched multi-key launch (Tier-1)
# and the c2a / DCF configs alternated.  Usage: bash tools/ab_walk_prio.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:?tag}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
OUT=gpurun_out/ab_${T}.log
: > $OUT
DPF_AMD_LIB=$(libof wp) timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_configs_gpu.py tests/test_kernels_gpu.py tests/test_api_gpu.py tests/test_dcf.py -k "c2 or points or seeds or walk or evaluate_at or apply or dcf" > gpurun_out/t_${T}_wp.log 2>&1 || { echo "wp tests rc=$?"; tail -20 gpurun_out/t_${T}_wp.log; exit 1; }
echo "wp tests: $(tail -1 gpurun_out/t_${T}_wp.log)" | tee -a $OUT
for rep in 1 2 3; do
  for v in main wp; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u tools/bench_configs.py --only c2 --c2-batched-only > gpurun_out/ab_${T}_c2_${v}.jsonl 2>&1 || { echo "c2 rc=$?"; tail gpurun_out/ab_${T}_c2_${v}.jsonl; exit 1; }
    echo "c2 $v $rep $(tail -1 gpurun_out/ab_${T}_c2_${v}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['tier1_multi_key_ms'],4), round(d['tier1_multi_key_lds_frac'],3))")" | tee -a $OUT
  done
done
echo done
