#!/bin/bash
# Many-query scans over wide rows: the Four-Russians kernels' slice-major,
# XCD-local order (DPF_SCAN_M4_SLICE_MAJOR) and the grid floor divided by the
# row's slices (DPF_SCAN_GRID_WIDE) against the default: tests per variant,
# then the grid's wide rows at Q = 10 / 100 and c4 at Q = 16 / 64 / 100
# alternated, and a FETCH pass of the 16 KiB Q = 100 scan.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06k}
VARS=${VARS:-"main m4sm gwide both"}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
for v in $VARS; do
  DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_pir_grid_gpu.py tests/test_api_gpu.py tests/test_multidevice_gpu.py -k "inner_product or grid or record_width or pir_database or sharded or forced_peer" > gpurun_out/t_${T}_$v.log 2>&1 || { echo "$v tests rc=$?"; tail -20 gpurun_out/t_${T}_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_${T}_$v.log)"
done
for rep in 1 2; do
  for v in $VARS; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u tools/bench_configs.py --only pirgrid --grid 2048,16384:65536,1048576:10,100 --reps 6 > gpurun_out/ab_${T}_${v}_${rep}.jsonl 2>&1 || { echo "$v rc=$?"; tail gpurun_out/ab_${T}_${v}_${rep}.jsonl; exit 1; }
    DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u tools/bench_configs.py --only c4q --c4q-queries 16,64,100 --no-ab --reps 6 > gpurun_out/ab_${T}_c4_${v}_${rep}.jsonl 2>&1 || { echo "$v c4 rc=$?"; exit 1; }
    echo "$v $rep $(tail -1 gpurun_out/ab_${T}_${v}_${rep}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print([(r['records']>>16, r['avg_bytes'], r['batch'], round(r['scan_ms'],3)) for r in d['rows']])") $(tail -1 gpurun_out/ab_${T}_c4_${v}_${rep}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v,3) for k,v in d.items() if k.endswith('_ms')})")"
  done
done
for v in $VARS; do
  DPF_AMD_LIB=$(libof $v) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_$v -o f --output-format csv -- python3 tools/bench_configs.py --only pirgrid --grid 16384:1048576:100 --reps 2 > gpurun_out/pmc_${T}_$v.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
done
echo done
