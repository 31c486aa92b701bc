#!/bin/bash
# Determinism of the many-query scan per library variant (GPU box).
for v in "$@"; do
  if [ "$v" = main ]; then export DPF_AMD_LIB=; else
    export DPF_AMD_LIB=$PWD/distributed_point_functions_amd/_native/var_$v/libdpf_amd.so; fi
  timeout -k 10 200 python -u tools/diag_scan_determinism.py > gpurun_out/diag_$v.log 2>&1 || { echo "$v rc=$?"; tail -3 gpurun_out/diag_$v.log; exit 1; }
  echo "$v: $(grep '^q 64' gpurun_out/diag_$v.log)"
done
