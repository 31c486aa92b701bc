#!/bin/bash
# A/B of the batched EvaluateAt kernel (c2) across library variants (GPU box).
for v in "$@"; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 200 python -u tools/bench_configs.py --only c2 --c2-batched-only --reps 8 \
    > gpurun_out/ab_c2_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_c2_$v.log; exit 1; }
  tail -1 gpurun_out/ab_c2_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['tier1_multi_key_ms'], 3), 'ms')"
done
