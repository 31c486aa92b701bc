#!/bin/bash
# Wave-uniform walk levels of KExpand computed by lane 0 alone and broadcast
# (var_uw1, the c5 TU built from commit "KExpand: wave-uniform walk levels
# computed by one lane") against the main build: parity of the variant
# (forced shapes, configs, c5 all-leaf digests), then the c5 bench alternated.
set -o pipefail
mkdir -p gpurun_out
V=$PWD/distributed_point_functions_amd/_native/var_uw1/libdpf_amd.so
DPF_AMD_LIB=$V timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_fullsize_gpu.py tests/test_kernels_gpu.py tests/test_configs_gpu.py \
  > gpurun_out/t_r04r.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_r04r.log; exit 1; }
echo "uw1 tests: $(tail -n 1 gpurun_out/t_r04r.log)"
for v in main uw1 main uw1 main uw1; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else export DPF_AMD_LIB=$V; fi
  timeout -k 10 200 python -u bench.py --skip-pir --skip-cpu-baseline --steps 10 --warmup 2 \
    > gpurun_out/ab_c5_r04r_$v.log 2>&1 || { echo "c5 $v failed"; tail -3 gpurun_out/ab_c5_r04r_$v.log; exit 1; }
  tail -n 1 gpurun_out/ab_c5_r04r_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$v', 'G leaves/s=%.3f' % (d['value']/1e9), 'kernel_ms=%.2f' % r['kernel_ms'], 'frac=%.4f' % r['frac'])"
done
