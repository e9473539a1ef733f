#!/bin/bash
# Round-3: z-chunk tuner: parity (tune then step == plain stepping == oracle), then the
# default bench (tuned) and the same with --no-tune.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tune.py > gpurun_out/r03l_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03l_tests.log; [ $rc -ne 0 ] && exit $rc
MNL_TUNE_VERBOSE=1 timeout -k 10 400 python bench.py > gpurun_out/r03l_bench.json 2> gpurun_out/r03l_bench.err || exit $?
timeout -k 10 400 python bench.py --no-tune > gpurun_out/r03l_bench_notune.json 2> gpurun_out/r03l_bench_notune.err || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/r03l_bench.json", "gpurun_out/r03l_bench_notune.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["config"].get("zchunk_tuned"),
          {k: (v["ms_per_step"], v.get("zchunk_tuned")) for k, v in (d.get("configs") or {}).items()})
PY
