#!/bin/bash
# Round 6: the two-step footprint prototype (tools/micro/tb2w.hip) on the GPU: parity + timing
# of each binary given, then FETCH_SIZE / WRITE_SIZE passes (separate runs) of the last one.
#   gpurun -- 'bash tools/gpu_tb2w.sh "tb2w_b0 512 48" "tb2w_b1 512 48"'
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tb2w
last=""
for spec in "$@"; do
  set -- $spec
  bin=$1; shift
  echo "=== $bin $*"
  timeout -k 10 120 tools/micro/bin/$bin "$@" || exit $?
  last="$bin $*"
done
[ -n "$PMC" ] || exit 0
set -- $last
bin=$1; shift
tag=${bin}_$(echo "$*" | tr ' ' '_')
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tb2w/${tag}_stats -o run --output-format csv -- tools/micro/bin/$bin "$@" > gpurun_out/tb2w/${tag}_stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tb2w/${tag}_fetch -o run --output-format csv -- tools/micro/bin/$bin "$@" > gpurun_out/tb2w/${tag}_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tb2w/${tag}_write -o run --output-format csv -- tools/micro/bin/$bin "$@" > gpurun_out/tb2w/${tag}_write.log 2>&1 || exit $?
echo "pmc done: $tag"
