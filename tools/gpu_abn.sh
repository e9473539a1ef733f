#!/bin/bash
# Parity subset for the default library, then alternating bench processes of the default
# library and the variants in $VARIANTS (MNL_LIB_VARIANT), for the 512^3 waveguide and the
# vacuum headline; one summary line per run (step ms, tile-kernel launch ms).
#   VARIANTS="a b" REPS=3 bash tools/gpu_abn.sh
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-x}" != none ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_fullsize.py} > gpurun_out/abn_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/abn_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for wl in "" "--vacuum"; do
  for rep in $(seq ${REPS:-3}); do
    for v in base $VARIANTS; do
      if [ "$v" = base ]; then unset MNL_LIB_VARIANT; else export MNL_LIB_VARIANT=$v; fi
      timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-extra $wl > gpurun_out/abn_$v.log 2>&1 || exit $?
      python - "$v $wl" gpurun_out/abn_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:14s}: {d['ms_per_step']:.4f} ms/step  tile {r['avg_launch_ms']:.4f}", flush=True)
PY
    done
  done
done
