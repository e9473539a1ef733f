#!/bin/bash
# Round-3: does the combined tile kernel's SGPR pressure slow each body?  Body-class timing
# (host mask) with the production library vs libraries compiled with that body only,
# alternating processes; then in-process A/B of the x-coefficient hoist (VAR 8 / 16).
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2 3; do
  for pair in "1 lean1" "2 ax1" "4 ax2"; do
    set -- $pair
    MNL_TILE_BODY_MASK=$1 timeout -k 10 120 python tools/body_time.py || exit $?
    MNL_TILE_BODY_MASK=$1 MNL_LIB_VARIANT=$2 timeout -k 10 120 python tools/body_time.py || exit $?
  done
done
V="MNL_TILE_VAR=0 MNL_TILE_VAR=8 MNL_TILE_VAR=16"
for wl in "" "--workload c2 --size 256"; do
  echo "== $wl"
  MNL_LIB_VARIANT=ab timeout -k 10 300 python tools/ab_inproc.py $V -- $wl > gpurun_out/r03q_ab.log 2>&1 || exit $?
  grep "ms/step" gpurun_out/r03q_ab.log
done
