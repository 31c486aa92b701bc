#!/bin/bash
# DCF kernels (gpurun): parity of both kernels, the DCF config bench.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dcf.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_dcf.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_dcf.log; exit 1; }
tail -1 gpurun_out/t_dcf.log
timeout -k 10 300 python -u tools/bench_configs.py --only dcf > gpurun_out/cfg_dcf.log 2>&1 || { echo "cfg rc=$?"; tail -5 gpurun_out/cfg_dcf.log; exit 1; }
tail -1 gpurun_out/cfg_dcf.log
