#!/bin/bash
# Round-3: parity subset for the default library (RS descriptors, OWNC, skipped B loads,
# multi-axis DIST 0), in-process A/B of the tile-kernel switches (variant library built with
# -DMNL_TILE_AB: MNL_TILE_VAR / MNL_NO_OWNC), per-body timing.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_fullsize.py tests/test_gpu_mp.py > gpurun_out/r03f_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03f_tests.log; [ $rc -ne 0 ] && exit $rc
V="MNL_TILE_VAR=0,MNL_NO_OWNC=0 MNL_TILE_VAR=1,MNL_NO_OWNC=0 MNL_TILE_VAR=2,MNL_NO_OWNC=0 MNL_TILE_VAR=4,MNL_NO_OWNC=0 MNL_TILE_VAR=0,MNL_NO_OWNC=1 MNL_TILE_VAR=7,MNL_NO_OWNC=1"
for wl in "" "--vacuum" "--workload c2 --size 256"; do
  echo "== $wl"
  MNL_LIB_VARIANT=ab timeout -k 10 300 python tools/ab_inproc.py $V -- $wl > gpurun_out/r03f_ab.log 2>&1 || exit $?
  grep "ms/step" gpurun_out/r03f_ab.log
done
timeout -k 10 300 python tools/tile_bodies.py > gpurun_out/r03f_tb_wg.log 2>&1 || exit $?
grep -E "^mask" gpurun_out/r03f_tb_wg.log
