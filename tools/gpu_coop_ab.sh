#!/bin/bash
# KExpandCoop variant check (gpurun): parity of each non-traced variant on the
# cooperative / forced-depth / batched tests, then tools/coop_trace.py on the
# traced ones.  bash tools/gpu_coop_ab.sh "qb2" "ct8 ct8q1 ct8q2"
mkdir -p gpurun_out
N=$PWD/distributed_point_functions_amd/_native
for v in $1; do
  DPF_AMD_LIB=$N/var_$v/libdpf_amd.so timeout -k 10 400 python -u -m pytest tests/test_fullsize_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "coop or forced or batched or c1" > gpurun_out/t_coop_$v.log 2>&1 || { echo "$v parity rc=$?"; tail -20 gpurun_out/t_coop_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/t_coop_$v.log)"
done
for v in $2; do
  for w in ${3:-c1}; do
    [ -f $N/var_$v/libdpf_amd.so ] || continue
    DPF_AMD_LIB=$N/var_$v/libdpf_amd.so timeout -k 10 200 python -u tools/coop_trace.py $w > gpurun_out/coop_trace_${v}_$w.log 2>&1 || { echo "$v $w rc=$?"; tail -5 gpurun_out/coop_trace_${v}_$w.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/coop_trace_${v}_$w.log)"
  done
done
