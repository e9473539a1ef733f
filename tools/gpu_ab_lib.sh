#!/bin/bash
# Parity subset for the default library, then alternate bench runs of the default
# library and a variant (MNL_LIB_VARIANT) -- one summary line per run.
#   VARIANT=<name> REPS=3 bash tools/gpu_ab_lib.sh
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_fullsize.py} > gpurun_out/ablib_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ablib_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in $(seq ${REPS:-3}); do
  for v in base $VARIANT; do
    if [ "$v" = base ]; then unset MNL_LIB_VARIANT; else export MNL_LIB_VARIANT=$v; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-extra ${BENCH_ARGS} > gpurun_out/ablib_$v.log 2>&1 || exit $?
    python - "$v" gpurun_out/ablib_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]; g = r.get("general_kernel", {})
print(f"{sys.argv[1]}: {d['ms_per_step']:.4f} ms/step  lean {r['avg_launch_ms']:.4f}  general {g.get('avg_launch_ms', 0):.4f}")
PY
  done
done
