#!/bin/bash
# Scan-kernel variant check (gpurun): parity of each variant library on the
# scan tests, then the c4 many-query A/B.  Variants: tools/build_variants.py.
#   bash tools/gpu_scan_ab.sh <queries> v1 v2 ...
QS=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  [ "$v" = main ] && continue
  DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so timeout -k 10 400 \
    python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "inner_product or scan or c4" > gpurun_out/t_scan_$v.log 2>&1 || { echo "$v parity rc=$?"; tail -20 gpurun_out/t_scan_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/t_scan_$v.log)"
done
bash tools/ab_c4q.sh $QS main "$@"
