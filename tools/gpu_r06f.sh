#!/bin/bash
# c4/8 HandleRequest anatomy: host phase marks and a kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/pir_hr_probe.py --log-n 23 --queries 1 --reps 30 > gpurun_out/hr23_r06f.log 2>&1 || exit 1
DPF_AMD_TRACE_HOST=1 timeout -k 10 120 python -u tools/pir_hr_probe.py --log-n 23 --queries 1 --reps 5 > gpurun_out/hr23_trace_r06f.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/hr23k_r06f -o k --output-format csv -- python3 tools/pir_hr_probe.py --log-n 23 --queries 1 --reps 30 > gpurun_out/hr23k_r06f.log 2>&1 || exit 1
tail -2 gpurun_out/hr23_r06f.log
echo done
