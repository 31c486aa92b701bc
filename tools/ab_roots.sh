#!/bin/bash
# A/B of the roots stage of large expansions (DPF_AMD_EXPAND_ROOTS=0 vs the
# default) on one box: the parity tests of the stage and of c5 at full size,
# then c5 bench lines alternated.  Usage: bash tools/ab_roots.sh <tag> [rounds]
set -o pipefail
TAG=${1:?tag}
ROUNDS=${2:-3}
export TMPDIR=/tmp
mkdir -p gpurun_out
LOG=gpurun_out/ab_roots_${TAG}.log
timeout -k 10 500 python -u -m pytest tests/test_fullsize_gpu.py -x -q --timeout 400 \
  --timeout-method thread -k "roots or c5_full or production_depth or leaf_ranges" \
  > gpurun_out/ab_roots_tests_${TAG}.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/ab_roots_tests_${TAG}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab_roots_tests_${TAG}.log)" | tee $LOG
for i in $(seq 1 $ROUNDS); do
  for m in 0 1; do
    DPF_AMD_EXPAND_ROOTS=$m timeout -k 10 200 python -u bench.py --skip-pir --skip-cpu-baseline \
      --steps 10 --warmup 2 > gpurun_out/ab_roots_run.log 2>&1 \
      || { echo "bench rc=$?"; tail -20 gpurun_out/ab_roots_run.log; exit 1; }
    python - "$m" >> $LOG <<'EOF'
import json, sys
d = json.loads(open("gpurun_out/ab_roots_run.log").read().strip().splitlines()[-1])
r = d["roofline"]
print("roots=%s value=%.4e ms_per_step=%.3f kernel_ms=%.3f frac=%.4f" %
      (sys.argv[1] if sys.argv[1] != "1" else "default", d["value"], d["ms_per_step"],
       r["kernel_ms"], r["frac"]))
EOF
    tail -1 $LOG
  done
done
