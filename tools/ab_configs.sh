#!/bin/bash
# A/B of library variants on tools/bench_configs.py (GPU box):
#   bash tools/ab_configs.sh <configs> v1 v2 ...   ("main" = default build)
CFG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 300 python -u tools/bench_configs.py --only $CFG > gpurun_out/configs_$v.log 2>&1 || exit 1
  echo "== $v"; grep '^{' gpurun_out/configs_$v.log
done
