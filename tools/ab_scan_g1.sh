#!/bin/bash
# Wide-record masked scan (G = 1): loads in flight per lane (DPF_SCAN_G1_U)
# and the slice-major grid (DPF_SCAN_G1_SLICE_MAJOR) against the default:
# scan / width / grid tests on each variant library, then the grid's wide rows
# and c4 Q = 1 alternated, and a FETCH pass of the 16 KiB Q = 1 scan.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06h}
VARS=${VARS:-"main g1u16 g1sm g1both"}
libof() { if [ $1 = main ]; then echo distributed_point_functions_amd/_native/libdpf_amd.so; else echo distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; fi; }
for v in $VARS; do
  DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_pir_grid_gpu.py tests/test_api_gpu.py -k "inner_product or grid or record_width or pir_database" > gpurun_out/t_${T}_$v.log 2>&1 || { echo "$v tests rc=$?"; tail -20 gpurun_out/t_${T}_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_${T}_$v.log)"
done
for rep in 1 2; do
  for v in $VARS; do
    DPF_AMD_LIB=$(libof $v) timeout -k 10 300 python -u tools/bench_configs.py --only pirgrid --grid 2048,16384:1048576:1,2,10 --reps 10 > gpurun_out/ab_${T}_${v}_${rep}.jsonl 2>&1 || { echo "$v rc=$?"; tail gpurun_out/ab_${T}_${v}_${rep}.jsonl; exit 1; }
    echo "$v $rep $(tail -1 gpurun_out/ab_${T}_${v}_${rep}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print([(r['avg_bytes'], r['batch'], round(r['scan_ms'],3)) for r in d['rows']])")"
  done
done
for v in ${PMCVARS:-main g1sm g1both}; do
  DPF_AMD_LIB=$(libof $v) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_$v -o f --output-format csv -- python3 tools/bench_configs.py --only pirgrid --grid 16384:1048576:1 --reps 3 > gpurun_out/pmc_${T}_$v.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
done
echo done
