#!/bin/bash
# KExpand wave work queue for launches of a few block rounds
# (DPF_EXPAND_QUEUE) against the default: the expansion / incremental tests on
# the variant, then c3 and the c3-shaped probe alternated, and the c5 bench leg.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06n}
VARS="main q"
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
DPF_AMD_LIB=$(libof q) timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py tests/test_incremental_gpu.py tests/test_configs_gpu.py -k "not c5_full and not c4" > gpurun_out/t_${T}_q.log 2>&1 || { echo "q tests rc=$?"; tail -20 gpurun_out/t_${T}_q.log; exit 1; }
echo "q: $(tail -1 gpurun_out/t_${T}_q.log)"
for rep in 1 2; do
  for v in $VARS; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u tools/c3_expand_probe.py --roots 15,16,17 --depths 0 > gpurun_out/ab_${T}_probe_${v}_${rep}.log 2>&1 || { echo "probe rc=$?"; exit 1; }
    DPF_AMD_LIB=$(libof $v) timeout -k 10 200 python -u tools/bench_configs.py --only c3 > gpurun_out/ab_${T}_c3_${v}_${rep}.jsonl 2>&1 || { echo "c3 rc=$?"; exit 1; }
    echo "$v $rep $(grep roots gpurun_out/ab_${T}_probe_${v}_${rep}.log | awk '{print $2, $5}' | tr '\n' ' ') c3 $(tail -1 gpurun_out/ab_${T}_c3_${v}_${rep}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['device_out_ms_total'],3), d['device_out_ms_per_level'][4:8])")"
  done
done
for v in $VARS; do
  DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u bench.py --skip-pir --skip-cpu-baseline --steps 10 > gpurun_out/ab_${T}_c5_${v}.log 2>&1 || { echo "c5 rc=$?"; exit 1; }
  echo "$v c5 $(tail -1 gpurun_out/ab_${T}_c5_${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), round(d['roofline']['frac'],4))")"
done
