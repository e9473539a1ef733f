#!/bin/bash
# One GPU session: parity tests, smoke, bench; stops at the first crash/timeout.
# Exit codes 0/1 from pytest (pass / test failures) continue; anything else stops.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  return $rc
}
MODE=${1:-all}
step pytest_gpu 600 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS}
rc=$?; [ $rc -gt 1 ] && exit $rc
[ "$MODE" = tests ] && exit 0
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench256 300 python bench.py --size 256 --steps 40 --warmup 5 --no-cpu || exit $?
step bench512 600 python bench.py --steps 60 --warmup 10 || exit $?
exit 0
