set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
sha256sum distributed_point_functions_amd/_native/libdpf_amd.so > gpurun_out/lib_r06a.sha
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fullsize_gpu.py -k "forced_depth or depth6" tests/test_incremental_gpu.py > gpurun_out/t_r06a_new.log 2>&1 || { echo "new tests rc=$?"; tail -40 gpurun_out/t_r06a_new.log; exit 1; }
tail -1 gpurun_out/t_r06a_new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r06a.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/t_r06a.log; exit 1; }
tail -1 gpurun_out/t_r06a.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06a.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke_r06a.log; exit 1; }
tail -1 gpurun_out/smoke_r06a.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r06a.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_r06a.log; exit 1; }
tail -1 gpurun_out/bench_r06a.log | cut -c1-400
DPF_AMD_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --skip-cpu-baseline > gpurun_out/bench_r06a_gloo2.log 2>&1 || { echo "gloo2 rc=$?"; tail -20 gpurun_out/bench_r06a_gloo2.log; exit 1; }
tail -1 gpurun_out/bench_r06a_gloo2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('library_multi_device'))[:1500]); print(d['value'], d['pir']['correct'])"
echo done
