set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do for al in 16 128; do
timeout -k 10 300 python -u tools/bench_configs.py --only pirgrid --grid 2048,16384:1048576:1,10,100 --grid-align $al --reps 6 > gpurun_out/ab_align_${al}_${rep}.jsonl 2>&1 || exit 1
echo "$al $rep $(tail -1 gpurun_out/ab_align_${al}_${rep}.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print([(r['avg_bytes'], r['row_bytes'], r['batch'], round(r['scan_ms'],3)) for r in d['rows']])")"
done; done
for al in 16 128; do
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_align_$al -o f --output-format csv -- python3 tools/bench_configs.py --only pirgrid --grid 16384:1048576:1,100 --grid-align $al --reps 2 > gpurun_out/pmc_align_$al.log 2>&1 || exit 1
done
echo done
