#!/bin/bash
# Round-3: XCD-group tile queues (MNL_TILE_GROUPS): parity with the groups on, in-process
# A/B against the single queue on the three bench workloads.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
MNL_TILE_GROUPS=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/r03i_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03i_tests.log; [ $rc -ne 0 ] && exit $rc
V="MNL_TILE_GROUPS=1 MNL_TILE_GROUPS=8 MNL_TILE_GROUPS=24 MNL_TILE_GROUPS=4 MNL_TILE_GROUPS=20"
for wl in "" "--vacuum" "--workload c2 --size 256"; do
  echo "== $wl"
  timeout -k 10 300 python tools/ab_inproc.py $V -- $wl > gpurun_out/r03i_ab.log 2>&1 || exit $?
  grep "ms/step" gpurun_out/r03i_ab.log
done
