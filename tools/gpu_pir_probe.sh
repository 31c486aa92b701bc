#!/bin/bash
# HandleRequest in a torch process: phase times and a kernel trace (gpurun).
mkdir -p gpurun_out
DPF_AMD_TRACE_HOST=1 timeout -k 10 300 python -u tools/pir_hr_probe.py > gpurun_out/pir_probe.log 2> gpurun_out/pir_probe_trace.log || { echo "probe rc=$?"; tail -5 gpurun_out/pir_probe_trace.log; exit 1; }
cat gpurun_out/pir_probe.log
DPF_AMD_TRACE_HOST=1 timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 3 c4 > gpurun_out/pir_probe_cpp.log 2> gpurun_out/pir_probe_cpp_trace.log || { echo "cpp rc=$?"; exit 1; }
cat gpurun_out/pir_probe_cpp.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_hr -o hr -- python3 $GRAFT_REPO_ROOT/tools/pir_hr_probe.py --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_hr.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
