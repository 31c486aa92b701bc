#!/bin/bash
# Progress-ordered wave priority in the scans (variant `sp`, DPF_SCAN_PRIO=1)
# against the main build: the scan tests on the variant, then the c4 query
# sweep and the PIR grid alternated.  Usage: bash tools/ab_scan_prio.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:?tag}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
OUT=gpurun_out/ab_${T}.log
: > $OUT
DPF_AMD_LIB=$(libof sp) timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_pir_grid_gpu.py tests/test_api_gpu.py -k "scan or pir or inner_product" > gpurun_out/t_${T}_sp.log 2>&1 || { echo "sp tests rc=$?"; tail -20 gpurun_out/t_${T}_sp.log; exit 1; }
echo "sp tests: $(tail -1 gpurun_out/t_${T}_sp.log)" | tee -a $OUT
for rep in 1 2; do
  for v in main sp; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u tools/bench_configs.py --only c4q --no-ab > gpurun_out/ab_${T}_c4q_${v}.jsonl 2>&1 || { echo "c4q rc=$?"; tail gpurun_out/ab_${T}_c4q_${v}.jsonl; exit 1; }
    echo "c4q $v $rep $(tail -1 gpurun_out/ab_${T}_c4q_${v}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v, 3) for k, v in d.items() if k.endswith('_ms') and k[1:2].isdigit()})")" | tee -a $OUT
    DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u tools/bench_configs.py --only pirgrid --reps 5 --grid 256,2048,16384:1048576:1,10,100 > gpurun_out/ab_${T}_grid_${v}.jsonl 2>&1 || { echo "grid rc=$?"; tail gpurun_out/ab_${T}_grid_${v}.jsonl; exit 1; }
    echo "grid $v $rep $(tail -1 gpurun_out/ab_${T}_grid_${v}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print([(r['avg_bytes'], r['batch'], round(r['scan_ms'], 3)) for r in d['rows']])")" | tee -a $OUT
  done
done
echo done
