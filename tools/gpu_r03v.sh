#!/bin/bash
# Round-3: DFT work on a side stream beside the next step (one rank, fused): the DFT / flux
# parity tests and the fuzz families with flux planes, then the 4-plane flux bench with the
# side stream and with MNL_DFT_SYNC=1 (the DFT work on the stepping stream).
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
MNL_DFT_SIDE=1 timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dft.py tests/test_gpu_dft_fields.py tests/test_gpu_fuzz.py tests/test_gpu_mu.py \
  tests/test_gpu_sim_api.py tests/test_gpu_mp.py > gpurun_out/r03v_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03v_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  MNL_DFT_SIDE=$v timeout -k 10 300 python bench.py --flux 4 --no-cpu --no-extra > gpurun_out/r03v_flux_$v.json 2>/dev/null || exit $?
  python -c "import json; d=json.load(open('gpurun_out/r03v_flux_$v.json')); print('MNL_DFT_SIDE=$v', d['value'], d['ms_per_step'])"
done
