#!/bin/bash
# bench.py at N = 2 with gloo collectives, both ranks on the one GPU (a
# correctness rehearsal of the sharded data path, not a measurement), then
# the C++ c3 API with its std::vector floor.
mkdir -p gpurun_out
DPF_AMD_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --skip-cpu-baseline \
  > gpurun_out/bench_n2_gloo.log 2>&1 || { echo "n2 rc=$?"; tail -20 gpurun_out/bench_n2_gloo.log; exit 1; }
tail -1 gpurun_out/bench_n2_gloo.log | cut -c1-400
timeout -k 10 300 distributed_point_functions_amd/_native/cpp_api_bench 3 c3 > gpurun_out/cpp_c3_floor.log 2>&1 || { echo "c3 rc=$?"; exit 1; }
cat gpurun_out/cpp_c3_floor.log
