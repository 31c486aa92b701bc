#!/bin/bash
# Round 6: the PIR grid (tests, timings, a PMC profile of the 16 KiB scan) and
# PMC profiles of the c2 / c3 kernels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pir_grid_gpu.py > gpurun_out/t_r06b_grid.log 2>&1 || { echo "grid tests rc=$?"; tail -40 gpurun_out/t_r06b_grid.log; exit 1; }
tail -1 gpurun_out/t_r06b_grid.log
timeout -k 10 400 python -u tools/bench_configs.py --only pirgrid --reps 5 > gpurun_out/pirgrid_r06b.jsonl 2>&1 || { echo "pirgrid rc=$?"; tail -20 gpurun_out/pirgrid_r06b.jsonl; exit 1; }
echo "pirgrid ok"
PROF_SCRIPT=tools/bench_configs.py bash tools/profile_gpu.sh r06grid --only pirgrid --grid 16384:1048576:1,100 --reps 3 || exit 1
PROF_SCRIPT=tools/bench_configs.py bash tools/profile_gpu.sh r06c23 --only c2,c3 --reps 2 || exit 1
echo done
