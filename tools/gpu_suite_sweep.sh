mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r03s.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/gpu_tests_r03s.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03s.log
timeout -k 10 300 python -u tools/expand_sweep.py single > gpurun_out/sweep_single_r03s.log 2>&1 || { echo "sweep rc=$?"; tail -5 gpurun_out/sweep_single_r03s.log; exit 1; }
timeout -k 10 300 python -u tools/expand_sweep.py batched > gpurun_out/sweep_batched_r03s.log 2>&1 || { echo "sweep b rc=$?"; tail -5 gpurun_out/sweep_batched_r03s.log; exit 1; }
tail -3 gpurun_out/sweep_single_r03s.log
