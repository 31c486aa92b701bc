#!/bin/bash
# DCF kernel variants (gpurun): parity of each variant on tests/test_dcf.py,
# then the DCF config bench.  bash tools/gpu_dcf_ab.sh "main dq3w6 ..."
# (variants built with tools/build_variants.py k_walk.hip name:DEFS).
mkdir -p gpurun_out
N=$PWD/distributed_point_functions_amd/_native
for v in $1; do
  if [ "$v" = main ]; then LIB=$N/libdpf_amd.so; else LIB=$N/var_$v/libdpf_amd.so; fi
  DPF_AMD_LIB=$LIB timeout -k 10 400 python -u -m pytest tests/test_dcf.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_dcf_$v.log 2>&1 || { echo "$v tests rc=$?"; tail -30 gpurun_out/t_dcf_$v.log; exit 1; }
  DPF_AMD_LIB=$LIB timeout -k 10 300 python -u tools/bench_configs.py --only dcf > gpurun_out/cfg_dcf_$v.log 2>&1 || { echo "$v cfg rc=$?"; tail -5 gpurun_out/cfg_dcf_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/t_dcf_$v.log) | $(tail -1 gpurun_out/cfg_dcf_$v.log | cut -c1-400)"
done
