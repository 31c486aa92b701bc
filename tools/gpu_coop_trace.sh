#!/bin/bash
# KExpandCoop phase times (gpurun): tools/coop_trace.py on the traced variants.
mkdir -p gpurun_out
N=$PWD/distributed_point_functions_amd/_native
DPF_AMD_LIB=$N/var_ct8/libdpf_amd.so timeout -k 10 200 python -u tools/coop_trace.py c1 > gpurun_out/coop_trace_c1.log 2>&1 || { echo "c1 rc=$?"; tail -5 gpurun_out/coop_trace_c1.log; exit 1; }
DPF_AMD_LIB=$N/var_ct16/libdpf_amd.so timeout -k 10 200 python -u tools/coop_trace.py sel > gpurun_out/coop_trace_sel.log 2>&1 || { echo "sel rc=$?"; tail -5 gpurun_out/coop_trace_sel.log; exit 1; }
tail -1 gpurun_out/coop_trace_c1.log
tail -1 gpurun_out/coop_trace_sel.log
