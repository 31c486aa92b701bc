#!/bin/bash
# Round 5: PIR request path after the per-group restructure (one packed key
# upload, one allocation, shared fold slots, fold into mapped host memory):
# parity of the scan / PIR / sharded tests, then HandleRequest timings on 1
# and 8 shards of one GPU (plain and forced-peer), the 2^23-record shard as
# the N = 8 per-rank proxy, and the slots A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_multidevice_gpu.py \
  tests/test_configs_gpu.py tests/test_cuckoo_pir.py tests/test_api_gpu.py tests/test_wire_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -k "inner_product or scan or pir or c4 or shard or peer or cuckoo or request" \
  > gpurun_out/t_r05b.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_r05b.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_r05b.log)"
probe() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python -u tools/pir_hr_probe.py "$@" > gpurun_out/hr_${tag}_r05b.log 2>&1 \
    || { echo "probe $tag rc=$?"; tail gpurun_out/hr_${tag}_r05b.log; exit 1; }
  echo "$tag: $(grep '^Q=' gpurun_out/hr_${tag}_r05b.log | tr '\n' ' ')"
}
probe s1 --queries 1,8,64 --reps 10
probe s8 --queries 1,8,64 --reps 10 --devices 0,0,0,0,0,0,0,0
probe s8fp --queries 1,8,64 --reps 10 --devices 0,0,0,0,0,0,0,0 --force-peer
probe n23 --queries 1,8 --reps 20 --log-n 23
DPF_AMD_SCAN_SLOTS=0 probe n23noslots --queries 1,8 --reps 20 --log-n 23
probe n23b --queries 1,8 --reps 20 --log-n 23
DPF_AMD_SCAN_SLOTS=0 probe s1noslots --queries 1,8 --reps 10
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/hrtrace_n23_r05b -o tr \
  --output-format csv -- python3 tools/pir_hr_probe.py --queries 1 --reps 5 --log-n 23 \
  > gpurun_out/hrtrace_n23_r05b.log 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/hrtrace_s8_r05b -o tr \
  --output-format csv -- python3 tools/pir_hr_probe.py --queries 1 --reps 5 --devices 0,0,0,0,0,0,0,0 \
  > gpurun_out/hrtrace_s8_r05b.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo done
