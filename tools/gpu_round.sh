#!/bin/bash
# One box, the round's evidence for the current build: the whole GPU suite
# and smoke(), the N = 1 bench line, the reference's published experiment
# workloads, and the rocprofv3 profile of the bench (trace pass + separate
# PMC passes, tools/profile_gpu.sh) that the bench line's `traffic` reads.
# Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/t_${TAG}.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/t_${TAG}.log; exit 1; }
echo "gpu tests: $(tail -1 gpurun_out/t_${TAG}.log)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
  || { echo "smoke rc=$?"; tail gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_${TAG}.log 2>&1 \
  || { echo "bench rc=$?"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-300
timeout -k 10 600 python -u bench.py --experiments --steps 3 > gpurun_out/experiments_${TAG}.jsonl 2>&1 \
  || { echo "experiments rc=$?"; tail gpurun_out/experiments_${TAG}.jsonl; exit 1; }
tail -1 gpurun_out/experiments_${TAG}.jsonl
bash tools/profile_gpu.sh ${TAG} || exit 1
echo done
