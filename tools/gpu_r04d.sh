#!/bin/bash
# c5 A/B: the last AES round on the VALU (tools/experiments/
# gen_bs_last_round.py) — var_bslast: the tree pair's; var_bslast2: also the
# value-PRG pairs' — against the T-table build.  Bit-exactness on all 2^32
# leaves (subtree digests vs the oracle's) first, then the headline bench,
# alternated.
set -o pipefail
mkdir -p gpurun_out
var() { echo $PWD/distributed_point_functions_amd/_native/var_$1/libdpf_amd.so; }
for v in bslast bslast2; do
  DPF_AMD_LIB=$(var $v) timeout -k 10 400 python -u -m pytest -x -v --timeout 380 \
    --timeout-method thread tests/test_fullsize_gpu.py -k "c5" > gpurun_out/t_r04d_$v.log 2>&1 \
    || { echo "$v parity rc=$?"; tail -20 gpurun_out/t_r04d_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/t_r04d_$v.log)"
done
for v in main bslast bslast2 main bslast bslast2; do
  if [ "$v" = main ]; then L=; else L=$(var $v); fi
  DPF_AMD_LIB=$L timeout -k 10 200 python -u bench.py --skip-pir --skip-cpu-baseline --steps 10 \
    --warmup 2 > gpurun_out/ab_c5_$v.log 2>&1 || { echo "c5 $v failed"; tail -3 gpurun_out/ab_c5_$v.log; exit 1; }
  tail -1 gpurun_out/ab_c5_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$v', 'G leaves/s=%.3f' % (d['value']/1e9), 'kernel_ms=%.2f' % r['kernel_ms'], 'frac=%.3f' % r['frac'])"
done
