#!/bin/bash
# Headline bench re-check: tuned and untuned, headline only, and the one-step-call overhead.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --no-extra > gpurun_out/r03w_a.json || exit $?
timeout -k 10 200 python bench.py --no-cpu --no-extra --no-tune > gpurun_out/r03w_b.json || exit $?
timeout -k 10 200 python tools/step1_overhead.py || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/r03w_a.json", "gpurun_out/r03w_b.json"):
    d = json.load(open(f))
    print(f, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["tuned_zchunk_gen_cus"])
PY
