#!/bin/bash
# A/B of the many-query scan across library variants (GPU box):
#   bash tools/ab_c4q.sh <queries> v1 v2 ...   ("main" = the default build)
QS=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 200 python -u tools/bench_configs.py --only c4q --c4q-queries $QS --no-ab \
    > gpurun_out/ab_c4q_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_c4q_$v.log; exit 1; }
  tail -1 gpurun_out/ab_c4q_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$v', ' '.join('%s=%.2f' % (k, v) for k, v in d.items() if k.endswith('_ms')))"
done
