#!/bin/bash
# Round 5, first box: the GPU suite, the N = 1 bench line, the N = 2 launch
# rehearsal without torchrun (gloo, both ranks on the one GPU), and a kernel
# trace + host phase times of the c4 Q = 1 request on 1 and 8 shards of one
# GPU (the per-shard fixed cost).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/t_r05a.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/t_r05a.log; exit 1; }
echo "gpu tests: $(tail -1 gpurun_out/t_r05a.log)"
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r05a.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_r05a.log; exit 1; }
tail -1 gpurun_out/bench_r05a.log | cut -c1-400
DPF_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
  --cpu-seconds 4 > gpurun_out/bench_n2_gloo_r05a.log 2>&1 || { echo "n2 rc=$?"; tail -20 gpurun_out/bench_n2_gloo_r05a.log; exit 1; }
tail -1 gpurun_out/bench_n2_gloo_r05a.log | cut -c1-400
for D in 0 0,0,0,0,0,0,0,0; do
  tag=$(echo $D | tr -cd , | wc -c)
  DPF_AMD_TRACE_HOST=1 timeout -k 10 120 python -u tools/pir_hr_probe.py --queries 1,64 --reps 5 \
    --devices $D > gpurun_out/hr_s${tag}_r05a.log 2>&1 || { echo "probe rc=$?"; tail gpurun_out/hr_s${tag}_r05a.log; exit 1; }
  grep "^Q=" gpurun_out/hr_s${tag}_r05a.log
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/hrtrace_s${tag}_r05a -o tr \
    --output-format csv -- python3 tools/pir_hr_probe.py --queries 1 --reps 5 --devices $D \
    > gpurun_out/hrtrace_s${tag}_r05a.log 2>&1 || { echo "trace rc=$?"; exit 1; }
done
timeout -k 10 120 python -u tools/pir_hr_probe.py --queries 1,64 --reps 10 --log-n 23 \
  > gpurun_out/hr_n23_r05a.log 2>&1 && grep "^Q=" gpurun_out/hr_n23_r05a.log
