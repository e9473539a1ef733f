#!/bin/bash
# Baseline session: driver-style default bench (timed wall), vacuum headline, kernel stats.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03a}
s=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.err || exit $?
echo "default bench wall $(( $(date +%s) - s )) s"; cat gpurun_out/${TAG}_default.json | cut -c1-400
timeout -k 10 200 python bench.py --vacuum --no-extra --no-cpu > gpurun_out/${TAG}_vac.json || exit $?
cut -c1-300 gpurun_out/${TAG}_vac.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_vac -o run --output-format csv \
  -- python3 bench.py --vacuum --steps 20 --warmup 5 --no-cpu --no-extra > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
find gpurun_out/prof_${TAG}_vac -name "*kernel_stats*"
