#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (kernel times) -> gpurun_out/prof
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/prof
ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
  -- python3 bench.py $ARGS > gpurun_out/prof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 gpurun_out/prof/bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
