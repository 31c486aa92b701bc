#!/bin/bash
# Progress-ordered wave priority in KExpand (variants `prio`, DPF_EXPAND_PRIO=1:
# quarters; `prio2`, =2: geometric steps at 3/4, 7/8, 15/16)
# against the main build: expansion tests on the variant, then the c3-shaped
# probe, the c3 levels and the c5 bench leg, alternated.
# Usage: bash tools/ab_expand_prio.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:?tag}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
OUT=gpurun_out/ab_${T}.log
: > $OUT
for v in ${TESTED:-prio2}; do
  DPF_AMD_LIB=$(libof $v) timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py tests/test_incremental_gpu.py -k "not c5_full" > gpurun_out/t_${T}_$v.log 2>&1 || { echo "$v tests rc=$?"; tail -20 gpurun_out/t_${T}_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/t_${T}_$v.log)" | tee -a $OUT
done
for rep in 1 2; do
  for v in main prio prio2; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u tools/c3_expand_probe.py --roots 15,16,17 --depths 0 > gpurun_out/ab_${T}_probe_${v}_${rep}.log 2>&1 || { echo "probe rc=$?"; exit 1; }
    grep roots gpurun_out/ab_${T}_probe_${v}_${rep}.log | sed "s/^/probe $v $rep: /" | tee -a $OUT
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u tools/bench_configs.py --only c3 > gpurun_out/ab_${T}_c3_${v}_${rep}.jsonl 2>&1 || { echo "c3 rc=$?"; exit 1; }
    echo "c3 $v $rep $(tail -1 gpurun_out/ab_${T}_c3_${v}_${rep}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['device_out_ms_total'],3), d['device_out_ms_per_level'][4:10])")" | tee -a $OUT
  done
done
for rep in 1 2; do
  for v in main prio prio2; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u bench.py --skip-pir --skip-cpu-baseline --skip-library-multi-device --steps 10 --warmup 2 > gpurun_out/ab_${T}_c5_${v}.log 2>&1 || { echo "c5 $v rc=$?"; tail -20 gpurun_out/ab_${T}_c5_${v}.log; exit 1; }
    echo "c5 $v $rep $(tail -1 gpurun_out/ab_${T}_c5_${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline']['frac'],4))")" | tee -a $OUT
  done
done
echo done
