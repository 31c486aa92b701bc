#!/bin/bash
# Kernel durations of c1 (C++ EvaluateNext, 2^20 leaves) and a c4 Q = 1 / 8
# HandleRequest under rocprofv3 --kernel-trace (gpurun).
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c1 -o c1 -- $GRAFT_REPO_ROOT/distributed_point_functions_amd/_native/cpp_api_bench 10 c1 > $GRAFT_REPO_ROOT/gpurun_out/prof_c1.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_hr2 -o hr -- python3 $GRAFT_REPO_ROOT/tools/pir_hr_probe.py --reps 5 --queries 1,8 > $GRAFT_REPO_ROOT/gpurun_out/prof_hr2.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo done
