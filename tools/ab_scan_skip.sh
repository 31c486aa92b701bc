#!/bin/bash
# The opt-in scan that skips unselected records: its tests, then alternated
# timings against the default constant-time scan (c4 Q = 1, 2; the grid's
# wide records at Q = 1, 2) and a FETCH_SIZE pass of each at c4 Q = 1.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06c}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "scan or inner_product" > gpurun_out/t_${T}_skip.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_${T}_skip.log; exit 1; }
tail -1 gpurun_out/t_${T}_skip.log
for rep in 1 2; do
  for skip in 0 1; do
    DPF_AMD_SCAN_SKIP_UNSELECTED=$skip timeout -k 10 300 python -u tools/bench_configs.py --only c4q --c4q-queries 1,2 --no-ab --reps 20 > gpurun_out/ab_${T}_c4_s${skip}_${rep}.jsonl 2>&1 || { echo "c4q rc=$?"; exit 1; }
    DPF_AMD_SCAN_SKIP_UNSELECTED=$skip timeout -k 10 300 python -u tools/bench_configs.py --only pirgrid --grid 256,2048,16384:1048576:1,2 --reps 20 > gpurun_out/ab_${T}_grid_s${skip}_${rep}.jsonl 2>&1 || { echo "grid rc=$?"; exit 1; }
  done
done
for skip in 0 1; do
  DPF_AMD_SCAN_SKIP_UNSELECTED=$skip timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_skip${skip} -o f --output-format csv -- python3 tools/bench_configs.py --only c4q --c4q-queries 1 --no-ab --reps 3 > gpurun_out/pmc_${T}_skip${skip}.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
done
echo done
