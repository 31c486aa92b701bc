#!/bin/bash
# Depth-6 selection expansion (gpurun): forced-depth / batched parity, the
# batched sweep.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "forced_depth or batched" > gpurun_out/t_d6.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_d6.log; exit 1; }
tail -1 gpurun_out/t_d6.log
timeout -k 10 300 python -u tools/expand_sweep.py batched > gpurun_out/sweep_batched_d6.log 2>&1 || { echo "sweep rc=$?"; exit 1; }
grep mode gpurun_out/sweep_batched_d6.log | cut -c1-300
