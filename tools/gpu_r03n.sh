#!/bin/bash
# Round-3: polarization-chunk general kernel beside the tile kernel (MNL_TILE_GEN_CUS):
# parity with it on, in-process A/B of the CU split on C4.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
MNL_TILE_GEN_CUS=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_tune.py > gpurun_out/r03n_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03n_tests.log; [ $rc -ne 0 ] && exit $rc
V="MNL_TILE_GEN_CUS=0 MNL_TILE_GEN_CUS=32 MNL_TILE_GEN_CUS=64 MNL_TILE_GEN_CUS=96 MNL_TILE_GEN_CUS=128 MNL_TILE_GEN_CUS=160"
for wl in "--workload kerr --size 256" "--workload kerr --size 512"; do
  echo "== $wl"
  timeout -k 10 300 python tools/ab_inproc.py $V -- $wl > gpurun_out/r03n_ab.log 2>&1 || exit $?
  grep "ms/step" gpurun_out/r03n_ab.log
done
