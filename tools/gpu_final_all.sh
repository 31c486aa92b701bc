#!/bin/bash
# End-of-round GPU run (gpurun): tools/gpu_final.sh (suite, smoke, rocprofv3
# profile, bench line), then the C++ API configs and the DCF config bench.
TAG=${1:-r03}
bash tools/gpu_final.sh $TAG || exit 1
timeout -k 10 600 distributed_point_functions_amd/_native/cpp_api_bench 5 c1,c2,c2a,c3,c4 > gpurun_out/cpp_api_$TAG.log 2>&1 || { echo "cpp rc=$?"; tail -5 gpurun_out/cpp_api_$TAG.log; exit 1; }
cut -c1-200 gpurun_out/cpp_api_$TAG.log
timeout -k 10 300 python -u tools/bench_configs.py --only dcf > gpurun_out/cfg_dcf_$TAG.log 2>&1 || { echo "dcf rc=$?"; tail -5 gpurun_out/cfg_dcf_$TAG.log; exit 1; }
tail -1 gpurun_out/cfg_dcf_$TAG.log | cut -c1-300
