#!/bin/bash
# Round-3: narrow x-edge tiles (MNL_TILE_XEDGE = w): parity with w = 32 and 16, in-process A/B
# against 64-wide edge tiles on the bench workloads.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for w in 32 16; do
  MNL_TILE_XEDGE=$w timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/r03j_tests_$w.log 2>&1
  rc=$?; tail -1 gpurun_out/r03j_tests_$w.log; [ $rc -ne 0 ] && exit $rc
done
V="MNL_TILE_XEDGE=0 MNL_TILE_XEDGE=32 MNL_TILE_XEDGE=16"
for wl in "" "--vacuum" "--workload c2 --size 256" "--workload kerr --size 256" "--workload c5 --size 512"; do
  echo "== $wl"
  timeout -k 10 300 python tools/ab_inproc.py $V -- $wl > gpurun_out/r03j_ab.log 2>&1 || exit $?
  grep "ms/step" gpurun_out/r03j_ab.log
done
