#!/bin/bash
# c3's prefixes host-written into fine-grained device memory
# (DPF_AMD_PLACE_PREFIXES=1, the default since r06) against the pinned-slot
# copy + copy kernel (=0): the
# incremental tests with the option, then the c3 levels alternated.
# Usage: bash tools/ab_place_prefixes.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:?tag}
OUT=gpurun_out/ab_${T}.log
: > $OUT
DPF_AMD_PLACE_PREFIXES=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_incremental_gpu.py tests/test_configs_gpu.py -k "incremental or c3 or context or evaluate_until or prefix" > gpurun_out/t_${T}.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_${T}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_${T}.log)" | tee -a $OUT
for rep in ${REPS:-1 2 3}; do
  for m in ${ORDER:-0 1}; do
    DPF_AMD_PLACE_PREFIXES=$m timeout -k 10 200 python -u tools/bench_configs.py --only c3 > gpurun_out/ab_${T}_c3_$m.jsonl 2>&1 || { echo "c3 rc=$?"; exit 1; }
    echo "place=$m $rep $(tail -1 gpurun_out/ab_${T}_c3_$m.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['device_out_ms_total'],3), d['device_out_ms_per_level'][2:10])")" | tee -a $OUT
  done
done
echo done
