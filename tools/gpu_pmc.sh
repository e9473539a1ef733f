#!/bin/bash
# rocprofv3 profiling of the 512^3 bench: kernel-trace stats, then separate PMC
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass; --pmc never combined
# with sys/runtime traces).  Output -> gpurun_out/prof_<tag>/
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu --no-extra}
run() {  # run <name> <rocprof args...>
  local name=$1; shift
  echo "=== $name"
  timeout -k 10 400 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv \
    -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 $OUT/$name.log
  return $rc
}
run stats --kernel-trace --stats || exit $?
[ "$1" = stats ] && exit 0
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY || exit $?
run tcc --pmc TCC_HIT_sum TCC_MISS_sum || exit $?
run sq2 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH || exit $?
exit 0
