#!/bin/bash
# bench line with the opt-in skip leg, then the host-written level inputs
# (the applied host_write patch) A/B on c3 and the C++ API bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r06d.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_r06d.log; exit 1; }
tail -1 gpurun_out/bench_r06d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pir']; print(d['value'], d['roofline']['frac'], p['ms_per_query'], p['roofline']['frac'], json.dumps(p.get('skip_unselected'))[:600], json.dumps(p.get('handle_request'))[:300], json.dumps(p.get('handle_request_one_eighth'))[:300], d['library'])"
OUT=gpurun_out/ab_place_r06d.log
: > $OUT
for round in 1 2; do
  for v in new old; do
    if [ $v = old ]; then E="DPF_AMD_HOST_WRITE=0"; else E="DPF_AMD_HOST_WRITE=1"; fi
    echo "== $v round=$round" >> $OUT
    env $E timeout -k 10 200 ./distributed_point_functions_amd/_native/cpp_api_bench 6 2>&1 | grep -v amdgpu.ids | cut -c1-200 >> $OUT || { echo "cpp rc=$?"; tail -20 $OUT; exit 1; }
    env $E timeout -k 10 200 python -u tools/bench_configs.py --only c3 --no-ab 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c3 device_out_ms_total', round(d['device_out_ms_total'],3), d['device_out_ms_per_level'][3:8])" >> $OUT || { echo "c3 rc=$?"; tail -20 $OUT; exit 1; }
  done
done
cat $OUT | cut -c1-220
