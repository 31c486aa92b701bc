#!/bin/bash
# Round-4 profiles: one c3 run per EvaluateUntil strategy (host phases
# traced), rocprofv3 trace + PMC of c3 and of the Q = 64 scan, the 8-slice
# in-process rehearsal with the peer branches forced, and a D2H threshold A/B
# of the C++ EvaluateAt loop.
set -o pipefail
mkdir -p gpurun_out
for m in 0 1 0 1; do
  DPF_AMD_PREFIX_EXPAND=$((1 - m)) timeout -k 10 120 python -u tools/bench_configs.py --only c3 \
    > gpurun_out/c3_r04e_m$m.jsonl 2>&1 || { echo "c3 m$m failed"; exit 1; }
  tail -1 gpurun_out/c3_r04e_m$m.jsonl | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('expand_mode=$m host_ms=%.1f device_ms=%.2f per_level_dev=%s' % (d['host_out_ms_total'], d['device_out_ms_total'], d['device_out_ms_per_level'][5]))"
done
DPF_AMD_TRACE_HOST=1 timeout -k 10 120 python -u tools/bench_configs.py --only c3 --reps 1 \
  > gpurun_out/c3_r04e_trace.log 2>&1 || exit 1
ARGS="--only c3 --reps 2" timeout -k 10 900 bash tools/profile_configs.sh r04c3 || exit 1
timeout -k 10 900 bash tools/profile_configs.sh r04c4q || exit 1
timeout -k 10 300 python -u bench.py --in-process --devices 0,0,0,0,0,0,0,0 --force-peer --steps 3 \
  --warmup 1 > gpurun_out/bench_inproc8_r04e.log 2>&1 || { echo "inproc failed"; tail -5 gpurun_out/bench_inproc8_r04e.log; exit 1; }
tail -1 gpurun_out/bench_inproc8_r04e.log | cut -c1-400
for kb in 1024 64 1024 64; do
  DPF_AMD_D2H_DIRECT_KB=$kb timeout -k 10 120 distributed_point_functions_amd/_native/cpp_api_bench 5 c2 \
    > gpurun_out/cpp_c2_d2h$kb.log 2>&1 || exit 1
  echo "d2h_direct_kb=$kb $(tail -1 gpurun_out/cpp_c2_d2h$kb.log)"
done
