#!/bin/bash
# KPirScanM4<1> LDS/VALU query split (DPF_SCAN_M4_VALU_Q=16) against the
# default: the scan tests on each variant library, then Q = 48 / 56 / 64 on c4
# alternated (tools/build_variants.py k_pir.hip ... builds the variants).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06e}
VARS="main vq16s vq16v vq16w3 vq16vw3"
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
for v in $VARS; do
  DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "inner_product_each_scan_kernel or scan_kernels_agree_large" > gpurun_out/t_${T}_$v.log 2>&1 || { echo "$v tests rc=$?"; tail -20 gpurun_out/t_${T}_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_${T}_$v.log)"
done
for rep in 1 2; do
  for v in $VARS; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u tools/bench_configs.py --only c4q --c4q-queries 48,56,64 --no-ab --reps 10 > gpurun_out/ab_${T}_${v}_${rep}.jsonl 2>&1 || { echo "$v rc=$?"; tail gpurun_out/ab_${T}_${v}_${rep}.jsonl; exit 1; }
    echo "$v $rep $(tail -1 gpurun_out/ab_${T}_${v}_${rep}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v,3) for k,v in d.items() if k.endswith('_ms')})")"
  done
done
