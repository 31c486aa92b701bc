#!/bin/bash
# Round 5: register Four-Russians scan (KPirScanRF) — parity on every scan
# shape (forced), then the c4 many-query A/B (masked / LDS M4 / register RF).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "inner_product or scan" > gpurun_out/t_r05e.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/t_r05e.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_r05e.log)"
timeout -k 10 300 python -u tools/bench_configs.py --only c4q --c4q-queries 16,32,64,100 --reps 5 \
  > gpurun_out/c4q_rf_r05e.log 2>&1 || { echo "c4q rc=$?"; tail gpurun_out/c4q_rf_r05e.log; exit 1; }
tail -2 gpurun_out/c4q_rf_r05e.log
