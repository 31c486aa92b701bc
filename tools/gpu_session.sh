#!/bin/bash
# One GPU-box session (run through gpurun): the -m gpu suite, the c4q scan
# A/B, the bench line.  Stops at the first failing step.
TAG=${1:-r02}
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/${name}_$TAG.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 gpurun_out/${name}_$TAG.log
  [ $rc -eq 0 ] || exit $rc
}
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step c4q 300 python -u tools/bench_configs.py --only c4q
if [ -n "$VARIANT" ]; then
  DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$VARIANT/libdpf_amd.so \
    step c4q_$VARIANT 300 python -u tools/bench_configs.py --only c4q
fi
step bench 400 python -u bench.py
