#!/bin/bash
# A/B timing of library variants (GPU box): bash tools/ab_bench.sh v1 v2 ...
# "main" = the default build; others = _native/var_<v>/libdpf_amd.so.
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 200 python -u bench.py --skip-pir --skip-cpu-baseline --steps 5 --warmup 1 \
    > gpurun_out/bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e9, 3), 'G leaves/s', round(d['roofline']['kernel_ms'], 2), 'ms')"
done
