#!/bin/bash
# Expansion-kernel check (gpurun): forced-variant and full-size expansion
# parity, PIR tests, then the single and batched launch-size sweeps.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py tests/test_kernels_gpu.py tests/test_api_gpu.py tests/test_multidevice_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c5_full" > gpurun_out/t_coop_$TAG.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_coop_$TAG.log; exit 1; }
tail -1 gpurun_out/t_coop_$TAG.log
timeout -k 10 300 python -u tools/expand_sweep.py single > gpurun_out/sweep_single_$TAG.log 2>&1 || { echo "sweep rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/expand_sweep.py batched > gpurun_out/sweep_batched_$TAG.log 2>&1 || { echo "sweep rc=$?"; exit 1; }
grep mode gpurun_out/sweep_single_$TAG.log | cut -c1-250
grep mode gpurun_out/sweep_batched_$TAG.log | cut -c1-250
