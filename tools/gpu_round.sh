#!/bin/bash
# Full GPU validation of the current build (gpurun): the -m gpu suite, then
# the c3 check and the scan prefetch A/B (variants built beforehand with
# tools/build_variants.py).  Stops at the first failing step.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
bash tools/gpu_c3_check.sh $TAG || exit 1
if [ -n "$SCAN_AB" ]; then bash tools/ab_c4q.sh 64 $SCAN_AB || exit 1; fi
