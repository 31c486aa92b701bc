#!/bin/bash
# Evidence for the final library, part A: the whole GPU suite and smoke(),
# the N = 1 bench line, the two-rank gloo rehearsal (library_multi_device on
# one GPU, forced peer copies), and the rocprofv3 profile of the bench that
# the line's `traffic` is keyed on.
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
sha256sum distributed_point_functions_amd/_native/libdpf_amd.so > gpurun_out/lib_${TAG}.sha
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_${TAG}.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/t_${TAG}.log; exit 1; }
echo "gpu tests: $(tail -1 gpurun_out/t_${TAG}.log)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-300
DPF_AMD_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --skip-cpu-baseline > gpurun_out/bench_${TAG}_gloo2.log 2>&1 || { echo "gloo2 rc=$?"; tail -20 gpurun_out/bench_${TAG}_gloo2.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_gloo2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['library_multi_device']; print('gloo2', d['n_gpus'], m['correct'], m['c5']['ms_per_step'], m['c4']['ms_per_request'])"
bash tools/profile_gpu.sh ${TAG} || exit 1
echo done
