#!/bin/bash
# Round-3: z-chunk length sweep (in-process, MNL_ZCHUNK_STEP; 0 = the automatic choice) on
# the 256^3 configs, the C5 slab and the 512^3 waveguide.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V="MNL_ZCHUNK_STEP=0 MNL_ZCHUNK_STEP=8 MNL_ZCHUNK_STEP=12 MNL_ZCHUNK_STEP=16 MNL_ZCHUNK_STEP=20 MNL_ZCHUNK_STEP=24 MNL_ZCHUNK_STEP=32 MNL_ZCHUNK_STEP=48"
for wl in "--workload c2 --size 256" "--workload kerr --size 256" "--workload c5 --size 512" ""; do
  echo "== $wl"
  MNL_TILE_STATS=1 timeout -k 10 300 python tools/ab_inproc.py $V -- $wl > gpurun_out/r03k_ab.log 2>&1 || exit $?
  grep -E "ms/step|^tile: " gpurun_out/r03k_ab.log | uniq
done
