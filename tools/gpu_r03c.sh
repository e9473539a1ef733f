#!/bin/bash
# Round-3: PMC passes of the tile kernel (512^3 waveguide, 512^3 vacuum) and a
# kernel trace of C2 256^3 (per-launch timeline).  Stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAG=r03c_wg bash tools/gpu_pmc.sh || exit $?
TAG=r03c_vac BENCH_ARGS="--vacuum --steps 10 --warmup 2 --no-cpu --no-extra" bash tools/gpu_pmc.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r03c_c2 -o run --output-format csv \
  -- python3 bench.py --workload c2 --size 256 --steps 20 --warmup 5 --no-cpu --no-extra \
  > gpurun_out/r03c_c2.log 2>&1 || exit $?
exit 0
