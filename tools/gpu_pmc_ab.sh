#!/bin/bash
# A/B PMC passes (FETCH_SIZE, TCC hit/miss) of the bench under two env settings.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
ARGS="--steps 6 --warmup 2 --no-cpu"
for v in ${VARIANTS:-"X=0"}; do
  for pm in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS"; do
    tag="$v.$(echo $pm | cut -d' ' -f1)"
    echo "=== $tag"
    env $v timeout -k 10 300 rocprofv3 --pmc $pm -d $OUT/$tag -o run --output-format csv \
      -- python3 bench.py $ARGS > $OUT/$tag.log 2>&1 || exit $?
  done
done
exit 0
