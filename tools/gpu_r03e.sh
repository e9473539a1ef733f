#!/bin/bash
# Round-3: H-side material and Simulation-API GPU tests, then the per-body timing of
# tools/gpu_r03d.sh.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mu.py tests/test_gpu_sim_api.py -m gpu -v --timeout 300 --timeout-method thread -rf \
  > gpurun_out/r03e_pytest_mu.log 2>&1
rc=$?; tail -40 gpurun_out/r03e_pytest_mu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_r03d.sh
