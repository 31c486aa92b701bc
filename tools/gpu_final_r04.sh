#!/bin/bash
# Round-4 end-of-round run: tools/gpu_final.sh (the -m gpu suite, smoke(), the
# rocprofv3 profile of bench.py keyed to this library, the bench line), then
# every config through tools/bench_configs.py and the C++ API bench.
TAG=${1:-r04f}
set -o pipefail
bash tools/gpu_final.sh $TAG || exit 1
timeout -k 10 600 python -u tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err \
  || { echo "configs rc=$?"; tail -5 gpurun_out/configs_$TAG.err; exit 1; }
echo "configs: $(wc -l < gpurun_out/configs_$TAG.jsonl) lines"
timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 5 c1,c2,c2a,c3,c4 > gpurun_out/cpp_api_$TAG.log 2>&1 \
  || { echo "cpp api rc=$?"; tail -5 gpurun_out/cpp_api_$TAG.log; exit 1; }
echo "cpp api: $(grep -c '^{' gpurun_out/cpp_api_$TAG.log) lines"
