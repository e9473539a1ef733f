#!/bin/bash
# Round-3: per-call host overhead fix (fused geometry reused while fused, NaN guard cadence
# across calls): one-step-call overhead, then the whole GPU suite.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python tools/step1_overhead.py || exit $?
timeout -k 10 200 python tools/step1_overhead.py --size 256 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf \
  > gpurun_out/r03s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03s_pytest.log; exit $rc
