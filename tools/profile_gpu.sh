#!/bin/bash
# Profiling recipe run on the GPU box.
# Usage: bash tools/profile_gpu.sh <tag> [bench args...]
#        PROF_SCRIPT=tools/bench_configs.py bash tools/profile_gpu.sh <tag> <its args...>
# Trace pass first, then one PMC pass per counter group (never combined with
# tracing).  Stops at the first abnormal exit (fault / abort / timeout).
TAG=${1:-r01}; shift
ARGS=${@:-"--steps 3 --warmup 1 --skip-cpu-baseline"}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# the profiled library: bench.py trusts PMC traffic only for this exact build
sha256sum ${DPF_AMD_LIB:-distributed_point_functions_amd/_native/libdpf_amd.so} | cut -d" " -f1 > $OUT/library.sha256
run() {  # name, timeout, rocprof args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 ${PROF_SCRIPT:-bench.py} $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
run trace 400 --kernel-trace --stats
run pmc_fetch 400 --pmc FETCH_SIZE
run pmc_write 400 --pmc WRITE_SIZE
run pmc_sq 400 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS
run pmc_sq2 240 --pmc SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
run pmc_grbm 400 --pmc GRBM_GUI_ACTIVE GRBM_COUNT
exit 0
