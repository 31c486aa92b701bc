#!/bin/bash
# A/B of the sharded HandleRequest's fixed cost on one box: the whole
# GPU suite, then pir_hr_probe.py alternated between the default (selection
# key host-written into fine-grained VRAM, fold slots kept zeroed by the
# fold) and DPF_AMD_HOST_WRITE=0 DPF_AMD_FOLD_CLEAR=0 (copy kernel + memset).
# Usage: bash tools/ab_hr.sh <tag>
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/ab_hr_${TAG}.log
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_hr_tests_${TAG}.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/ab_hr_tests_${TAG}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_hr_tests_${TAG}.log)" | tee $OUT
for round in 1 2; do
  for v in new old; do
    if [ $v = old ]; then E="DPF_AMD_HOST_WRITE=0 DPF_AMD_FOLD_CLEAR=0"; else E=""; fi
    for n in 23 26; do
      echo "== $v log_n=$n round=$round" >> $OUT
      env $E timeout -k 10 200 python -u tools/pir_hr_probe.py --log-n $n --queries 1,8 --reps 30 >> $OUT 2>&1 \
        || { echo "probe rc=$?"; tail -20 $OUT; exit 1; }
    done
  done
done
echo "== force-peer 8 shards" >> $OUT
timeout -k 10 200 python -u tools/pir_hr_probe.py --log-n 26 --queries 1,8 --reps 10 --devices 0,0,0,0,0,0,0,0 --force-peer >> $OUT 2>&1 \
  || { echo "probe rc=$?"; tail -20 $OUT; exit 1; }
grep -v "^\s*$" $OUT | tail -40
