#!/bin/bash
# A/B of the upload ring's H2D mode (DPF_AMD_UPLOAD: sdma = hipMemcpyAsync
# from the pinned slot, kernel_coherent = a copy kernel reading the slot
# mapped as fine-grained memory) on the C++ API configs and the c4/8
# request, alternated; then the GPU suite under the candidate mode.
# Usage: bash tools/ab_upload.sh <tag> <rounds> [suite]
set -o pipefail
TAG=${1:?tag}
ROUNDS=${2:?rounds}
export TMPDIR=/tmp
mkdir -p gpurun_out
LOG=gpurun_out/ab_upload_${TAG}.log
B=distributed_point_functions_amd/_native/cpp_api_bench
for i in $(seq 1 $ROUNDS); do
  for m in sdma kernel_coherent; do
    DPF_AMD_UPLOAD=$m timeout -k 10 200 $B 4 c1,c2,c2a,c3 > gpurun_out/up_$m.log 2>&1 \
      || { echo "cpp $m failed"; tail -5 gpurun_out/up_$m.log; exit 1; }
    DPF_AMD_UPLOAD=$m timeout -k 10 120 python -u tools/pir_hr_probe.py --log-n 23 --queries 1,8 \
      --reps 20 > gpurun_out/up_hr_$m.log 2>&1 || { echo "hr $m failed"; tail -5 gpurun_out/up_hr_$m.log; exit 1; }
    python3 - "$m" >> $LOG <<'PY'
import json, sys
m = sys.argv[1]
out = []
for line in open("gpurun_out/up_%s.log" % m):
    if line.startswith("{"):
        d = json.loads(line)
        out.append("%s=%s" % (d["config"], d.get("best_ms")))
hr = [l.strip() for l in open("gpurun_out/up_hr_%s.log" % m) if l.startswith("Q=")]
print(m, " ".join(out), "|", " ; ".join(hr))
PY
    tail -1 $LOG
  done
done
if [ "$3" = suite ]; then
  DPF_AMD_UPLOAD=kernel_coherent timeout -k 10 480 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/ab_upload_suite_${TAG}.log 2>&1 \
    || { echo "suite rc=$?"; tail -30 gpurun_out/ab_upload_suite_${TAG}.log; exit 1; }
  echo "suite (kernel_coherent): $(tail -1 gpurun_out/ab_upload_suite_${TAG}.log)" | tee -a $LOG
fi
