#!/bin/bash
# Round-3: tuner with the general-kernel split: tests, default bench tuned vs --no-tune.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tune.py tests/test_gpu_mp.py > gpurun_out/r03o_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03o_tests.log; [ $rc -ne 0 ] && exit $rc
MNL_TUNE_VERBOSE=1 timeout -k 10 400 python bench.py > gpurun_out/r03o_bench.json 2> gpurun_out/r03o_bench.err || exit $?
timeout -k 10 400 python bench.py --no-tune > gpurun_out/r03o_bench_notune.json 2> gpurun_out/r03o_bench_notune.err || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/r03o_bench.json", "gpurun_out/r03o_bench_notune.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["config"].get("tuned_zchunk_gen_cus"),
          {k: (v["ms_per_step"], v.get("tuned_zchunk_gen_cus")) for k, v in (d.get("configs") or {}).items()})
PY
grep "^tune" gpurun_out/r03o_bench.err
