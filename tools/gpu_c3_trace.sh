mkdir -p gpurun_out
DPF_AMD_TRACE_HOST=1 timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 2 c3 > gpurun_out/cpp_c3_b.log 2> gpurun_out/cpp_c3_trace_b.log || { echo "bench rc=$?"; tail -5 gpurun_out/cpp_c3_trace_b.log; exit 1; }
cat gpurun_out/cpp_c3_b.log
