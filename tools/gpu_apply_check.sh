#!/bin/bash
# Tier-2 host-overhead check (gpurun): EvaluateAndApply/DCF/API tests, the
# C++ API bench of c1-c3 with DPF_AMD_TRACE_HOST phase times, and a kernel
# trace of the c2 EvaluateAt loop.  Stops at the first failing step.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py tests/test_dcf.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_api_$TAG.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_api_$TAG.log; exit 1; }
tail -1 gpurun_out/t_api_$TAG.log
DPF_AMD_TRACE_HOST=1 timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 3 c1,c2,c2a,c3 > gpurun_out/cpp_$TAG.log 2> gpurun_out/cpp_trace_$TAG.log || { echo "bench rc=$?"; tail -20 gpurun_out/cpp_trace_$TAG.log; exit 1; }
cat gpurun_out/cpp_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$TAG -o c2 -- $GRAFT_REPO_ROOT/distributed_point_functions_amd/_native/cpp_api_bench 2 c2 > $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$TAG.log 2>&1 || { echo "prof rc=$?"; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$TAG -name "*stats*" | head
cd $GRAFT_REPO_ROOT
hipcc --offload-arch=gfx950 -O2 -o /tmp/malloc_async_repro tools/malloc_async_repro.cc || exit 1
for m in async async2 malloc; do
  timeout -k 10 200 /tmp/malloc_async_repro $m 3 > gpurun_out/malloc_repro_${m}_$TAG.log 2>&1; echo "repro $m rc=$?"; tail -1 gpurun_out/malloc_repro_${m}_$TAG.log
done
DPF_AMD_MALLOC_ASYNC=1 timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 3 c3 > gpurun_out/cpp_c3_mallocasync_$TAG.log 2>&1; echo "c3 mallocasync rc=$?"; tail -2 gpurun_out/cpp_c3_mallocasync_$TAG.log
