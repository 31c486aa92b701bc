hipcc --offload-arch=gfx950 -O2 -o /tmp/malloc_async_repro tools/malloc_async_repro.cc || exit 1
mkdir -p gpurun_out
for m in async malloc; do
  timeout -k 10 200 /tmp/malloc_async_repro $m 2 > gpurun_out/malloc_repro_${m}_b.log 2>&1; echo "repro $m rc=$?"; head -6 gpurun_out/malloc_repro_${m}_b.log; tail -1 gpurun_out/malloc_repro_${m}_b.log
done
