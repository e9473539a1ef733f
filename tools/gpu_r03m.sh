#!/bin/bash
# Round-3: multi-process slabs with the z-chunk tuner, and the 2-rank bench rehearsal
# (both ranks on one GPU over IPC) with tuning before the warm-up.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_mp.py > gpurun_out/r03m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03m_tests.log; [ $rc -ne 0 ] && exit $rc
MNL_TUNE_VERBOSE=1 MNL_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --size 256 --steps 10 \
  --warmup 2 --no-cpu > gpurun_out/r03m_bench2.json 2> gpurun_out/r03m_bench2.err || exit $?
cut -c1-300 gpurun_out/r03m_bench2.json; grep tune_zchunk gpurun_out/r03m_bench2.err
