#!/bin/bash
# PMC of the temporal-blocking prototype (tools/micro/tb2.hip): HBM bytes per launch of the
# 1-step and 2-step tile kernels (separate FETCH_SIZE / WRITE_SIZE passes).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tb2_pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tb2_pmc/stats -o run --output-format csv -- tools/micro/bin/tb2 512 64 6 > gpurun_out/tb2_pmc/stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tb2_pmc/fetch -o run --output-format csv -- tools/micro/bin/tb2 512 64 6 > gpurun_out/tb2_pmc/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tb2_pmc/write -o run --output-format csv -- tools/micro/bin/tb2 512 64 6 > gpurun_out/tb2_pmc/write.log 2>&1 || exit $?
grep -h "G cell-steps" gpurun_out/tb2_pmc/stats.log
