#!/bin/bash
# Wave priority in KPirScanM4 and the DCF kernel (main build: on) against a
# variant with both off (`off`: DPF_SCAN_M4_PRIO=0, DPF_DCF_PRIO=0): the scan
# and DCF tests on the main build, then the c4 query sweep and the DCF config
# alternated.  Usage: bash tools/ab_m4_dcf_prio.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:?tag}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
OUT=gpurun_out/ab_${T}.log
: > $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_dcf.py tests/test_configs_gpu.py -k "scan or dcf or c4" > gpurun_out/t_${T}.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_${T}.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_${T}.log)" | tee -a $OUT
for rep in 1 2 3; do
  for v in off main; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u tools/bench_configs.py --only c4q,dcf --no-ab --c4q-queries 16,32,64 > gpurun_out/ab_${T}_${v}.jsonl 2>&1 || { echo "cfg rc=$?"; tail gpurun_out/ab_${T}_${v}.jsonl; exit 1; }
    echo "$v $rep $(grep '^{' gpurun_out/ab_${T}_${v}.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    if d['config']=='c4q': print({k: round(v, 3) for k, v in d.items() if k.endswith('_ms') and k[1:2].isdigit()}, end=' ')
    if d['config']=='dcf': print('dcf', round(d['kernel_ms'], 4), end=' ')
")" | tee -a $OUT
  done
done
echo done
