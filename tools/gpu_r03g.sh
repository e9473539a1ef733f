#!/bin/bash
# Round-3 end-of-kernel-work measurements: the default bench as the driver runs it (wall time
# recorded), the vacuum headline, C5 at N=1, then rocprof kernel stats + PMC passes of the
# 512^3 waveguide and vacuum tile kernel (tools/gpu_pmc.sh).
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
s=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/r03g_default.json 2> gpurun_out/r03g_default.err || exit $?
echo "default bench wall $(( $(date +%s) - s )) s" | tee gpurun_out/r03g_wall.txt
timeout -k 10 200 python bench.py --vacuum --no-extra --no-cpu > gpurun_out/r03g_vac.json || exit $?
timeout -k 10 200 python bench.py --workload c5 --no-extra --no-cpu > gpurun_out/r03g_c5.json || exit $?
TAG=r03g_wg bash tools/gpu_pmc.sh || exit $?
TAG=r03g_vac BENCH_ARGS="--vacuum --steps 10 --warmup 2 --no-cpu --no-extra" bash tools/gpu_pmc.sh || exit $?
python - <<'PY'
import json
for f in ("r03g_default", "r03g_vac", "r03g_c5"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], d["config"]["model_fraction_of_peak"], r["avg_launch_ms"], r["frac"])
    for k, v in (d.get("configs") or {}).items():
        print("   ", k, v.get("value"), v.get("ms_per_step"), v.get("model_fraction_of_peak"))
PY
