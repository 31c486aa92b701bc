#!/bin/bash
# Whole -m gpu suite + C++ API configs (gpurun).  Stops at the first failure.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 600 distributed_point_functions_amd/_native/cpp_api_bench 5 c1,c2,c2a,c3,c4 > gpurun_out/cpp_$TAG.log 2>&1 || { echo "cpp rc=$?"; tail -5 gpurun_out/cpp_$TAG.log; exit 1; }
cut -c1-330 gpurun_out/cpp_$TAG.log
