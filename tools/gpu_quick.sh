#!/bin/bash
# Parity tests + 512^3 bench variants (env knobs) ; stops at first crash/timeout.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -f gpurun_out/steps.log
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 600 python -m pytest tests -m gpu -q -x -rf
rc=$?; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-"MNL_FUSED_BPC=1"}; do
  step "bench_$v" 300 env $v python bench.py --steps 40 --warmup 5 --no-cpu || exit $?
done
exit 0
