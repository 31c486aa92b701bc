#!/bin/bash
# rocprofv3 of tools/bench_configs.py runs (default: the many-query scan alone,
# c4 2^26 x 256 B, Q = 64; ARGS=... for another config):
# trace pass, then one PMC pass per counter group.
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
ARGS=${ARGS:-"--only c4q --c4q-queries 64 --no-ab --reps 3"}
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 tools/bench_configs.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run trace 300 --kernel-trace --stats
run pmc_fetch 300 --pmc FETCH_SIZE
run pmc_write 300 --pmc WRITE_SIZE
run pmc_sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD
run pmc_sq2 300 --pmc SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
