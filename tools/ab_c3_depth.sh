#!/bin/bash
# KExpand shape A/B: (1) c3's expansion at DFS depth 3 / 4 / 5 (variant `xd`,
# DPF_EXPAND_EXTRA_DEPTHS=1: 2^20 / 2^19 / 2^18 threads for c3's 2^16 prefix
# roots x 7 levels — four, two or one round of resident blocks), probe and
# the c3 levels; (2) the c5 kernel at 5 waves/SIMD (640-thread blocks) with 8
# or 4 staged leaves, and 4 staged leaves at 4 waves, against the main build.
# Usage: bash tools/ab_c3_depth.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:?tag}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
OUT=gpurun_out/ab_${T}.log
: > $OUT
for rep in 1 2; do
  DPF_AMD_LIB=$(libof xd) timeout -k 10 200 python -u tools/c3_expand_probe.py --roots 15,16,17 --depths 3,4,5 > gpurun_out/ab_${T}_probe_${rep}.log 2>&1 || { echo "probe rc=$?"; tail gpurun_out/ab_${T}_probe_${rep}.log; exit 1; }
  grep roots gpurun_out/ab_${T}_probe_${rep}.log | sed "s/^/probe $rep: /" | tee -a $OUT
done
for rep in 1 2; do
  for v in main w5s8 w5s4 w4s4; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u bench.py --skip-pir --skip-cpu-baseline --skip-library-multi-device --steps 10 --warmup 2 > gpurun_out/ab_${T}_c5_${v}.log 2>&1 || { echo "c5 $v rc=$?"; tail -20 gpurun_out/ab_${T}_c5_${v}.log; exit 1; }
    echo "c5 $v $rep $(tail -1 gpurun_out/ab_${T}_c5_${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],4))")" | tee -a $OUT
  done
done
echo done
