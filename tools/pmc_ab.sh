#!/bin/bash
# A/B of HBM traffic: one --pmc FETCH_SIZE pass and one WRITE_SIZE pass per variant
# VARIANTS="A=1 A=2" -> gpurun_out/pmcab_<i>_{fetch,write}/
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu}
i=0
for v in ${VARIANTS:-"X=0"}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    env $(echo $v | tr ',' ' ') timeout -k 10 -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmcab_${i}_$c -o run --output-format csv \
      -- python3 bench.py $ARGS > gpurun_out/pmcab_${i}_$c.log 2>&1 || exit $?
  done
  echo "$i $v"
  i=$((i+1))
done
