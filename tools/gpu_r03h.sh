#!/bin/bash
# Round-3: the whole GPU test suite as the driver runs it, smoke(), and the C5 8-rank
# decomposition rehearsed on one GPU (IPC transport).
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf \
  > gpurun_out/r03h_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03h_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03h_smoke.log 2>&1 || exit $?
cat gpurun_out/r03h_smoke.log
MNL_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 8 --workload c5 --size 128 --steps 10 \
  --warmup 2 --no-cpu > gpurun_out/r03h_c5_8ranks.json 2> gpurun_out/r03h_c5_8ranks.err || exit $?
cut -c1-400 gpurun_out/r03h_c5_8ranks.json
