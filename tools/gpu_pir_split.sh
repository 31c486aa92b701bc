#!/bin/bash
# PIR request pieces (gpurun): PIR tests, then C++ HandleRequest at c4 with
# DPF_AMD_PIR_SPLIT = 1 (one piece), automatic (2 from Q = 8) and 4.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multidevice_gpu.py tests/test_api_gpu.py tests/test_configs_gpu.py tests/test_cuckoo_pir.py tests/test_concurrency_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pir or shard or c4 or handle or cuckoo or thread" > gpurun_out/t_split.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/t_split.log; exit 1; }
tail -1 gpurun_out/t_split.log
for sp in 1 auto 4; do
  if [ $sp = auto ]; then unset DPF_AMD_PIR_SPLIT; else export DPF_AMD_PIR_SPLIT=$sp; fi
  timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 5 c4 > gpurun_out/c4split_$sp.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  echo "split=$sp: $(grep -o '"queries": [0-9]*, "best_ms": [0-9.]*' gpurun_out/c4split_$sp.log | tr '\n' ' ')"
done
