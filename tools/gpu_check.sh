#!/bin/bash
# A/B of the 512-child quad BFS level in KExpandCoop (main, DPF_COOP_QUAD_BFS=3)
# against the round-4 two quad levels (var_qb2): coop parity tests on main,
# then c1 and the c4/8 PIR request alternated.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py tests/test_multidevice_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "coop or expand or depth or shard" > gpurun_out/t_qb.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/t_qb.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t_qb.log)"
V=$PWD/distributed_point_functions_amd/_native/var_qb2/libdpf_amd.so
for v in main qb2 main qb2; do
  if [ $v = main ]; then unset DPF_AMD_LIB; else export DPF_AMD_LIB=$V; fi
  c1=$(timeout -k 10 120 python -u tools/bench_configs.py --only c1 --reps 20 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4f" % d["kernel_ms"], d["correct"])')
  hr=$(timeout -k 10 120 python -u tools/pir_hr_probe.py --queries 1 --reps 30 --log-n 23 2>/dev/null | grep "^Q=" | tr '\n' ' ')
  echo "$v c1_kernel_ms=$c1 | n23 $hr"
done
