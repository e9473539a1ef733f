#!/bin/bash
# Round-3 final check of the tree as the driver runs it: pytest -m gpu, smoke(), default bench.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf \
  > gpurun_out/r03r_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03r_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r_smoke.log 2>&1 || exit $?
cat gpurun_out/r03r_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r03r_bench.json 2> gpurun_out/r03r_bench.err || exit $?
cut -c1-400 gpurun_out/r03r_bench.json
