#!/bin/bash
# Evidence for the final library, part B: the secondary configs (c1-c3, c4
# many-query scans, DCF, cuckoo, the C++ API), the PIR grid, and the
# reference's published experiment workloads, and one rank's c5 slice at
# N = 1 / 2 / 4 / 8 (tools/c5_slice_probe.py).
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bench_configs.py --only c1,c2,c3,c4q,dcf,cuckoo,cpp > gpurun_out/configs_${TAG}.jsonl 2>&1 || { echo "configs rc=$?"; tail -20 gpurun_out/configs_${TAG}.jsonl; exit 1; }
echo "configs ok"
timeout -k 10 300 python -u tools/bench_configs.py --only pirgrid --reps 5 > gpurun_out/pirgrid_${TAG}.jsonl 2>&1 || { echo "pirgrid rc=$?"; exit 1; }
echo "pirgrid ok"
timeout -k 10 200 python -u tools/c5_slice_probe.py > gpurun_out/c5slice_${TAG}.log 2>&1 || { echo "c5 slices rc=$?"; tail gpurun_out/c5slice_${TAG}.log; exit 1; }
grep "^{" gpurun_out/c5slice_${TAG}.log
timeout -k 10 600 python -u bench.py --experiments --steps 3 > gpurun_out/experiments_${TAG}.jsonl 2>&1 || { echo "experiments rc=$?"; tail gpurun_out/experiments_${TAG}.jsonl; exit 1; }
tail -1 gpurun_out/experiments_${TAG}.jsonl
echo done
