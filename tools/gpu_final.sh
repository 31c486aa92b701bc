#!/bin/bash
# End-of-round GPU validation (gpurun): the -m gpu suite, smoke(), the
# rocprofv3 profile of the bench, and the bench line.  Stops at the first
# failing step.
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo "gpu tests rc=$?"; tail -5 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
bash tools/profile_gpu.sh $TAG || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
