#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_incremental_gpu.py tests/test_api_gpu.py tests/test_configs_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "incremental or ctx or evaluate_until or context or c3 or bookkeeping or prefix" > gpurun_out/t_r05i.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r05i.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_r05i.log)"
timeout -k 10 600 python -u bench.py --experiments --steps 3 > gpurun_out/experiments_r05i.jsonl 2>&1 \
  || { echo "experiments rc=$?"; tail gpurun_out/experiments_r05i.jsonl; exit 1; }
tail -1 gpurun_out/experiments_r05i.jsonl
