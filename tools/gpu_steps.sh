#!/bin/bash
# Run named GPU steps, each under its own time limit; stop at the first failure.
#   tools/gpu_steps.sh "name|seconds|command" ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name (limit ${to}s)"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
