#!/bin/bash
# c2 walk kernels after a change: walk/points/DCF parity tests, the C++ API
# c2/c2a bench and a kernel trace of the per-key EvaluateAt loop.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_api_gpu.py tests/test_dcf.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "walk or point or seeds or apply or dcf or c2 or evaluate_at" > gpurun_out/t_c2_$TAG.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_c2_$TAG.log; exit 1; }
tail -1 gpurun_out/t_c2_$TAG.log
timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 5 c2,c2a > gpurun_out/cpp_c2_$TAG.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/cpp_c2_$TAG.log; exit 1; }
cat gpurun_out/cpp_c2_$TAG.log
timeout -k 10 300 python -u tools/bench_configs.py --only c2 > gpurun_out/cfg_c2_$TAG.log 2>&1 || { echo "cfg rc=$?"; tail -5 gpurun_out/cfg_c2_$TAG.log; exit 1; }
tail -2 gpurun_out/cfg_c2_$TAG.log | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$TAG -o c2 -- $GRAFT_REPO_ROOT/distributed_point_functions_amd/_native/cpp_api_bench 2 c2,c2a > $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$TAG.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
