#!/bin/bash
# Parity tests (optional subset) then an in-process A/B of env variants on the 512^3 bench.
#   TESTS="tests/test_gpu_parity.py ..." VARIANTS="A=1 A=0" bash tools/gpu_ab.sh
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 200 --timeout-method thread \
    > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python -u tools/ab_inproc.py $VARIANTS -- ${BENCH_ARGS} > gpurun_out/ab.log 2>&1
rc=$?; tail -5 gpurun_out/ab.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu > gpurun_out/ab_bench.log 2>&1
  rc=$?; tail -1 gpurun_out/ab_bench.log | cut -c1-400; exit $rc
fi
