#!/bin/bash
# Round-3 session: new GPU tests, driver-style default bench (timed wall), vacuum
# headline, the old two-launch path for comparison, rocprof kernel stats.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03b}
T=${TESTS:-tests/test_gpu_dft_fields.py}
if [ "$T" != none ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread -rf \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
s=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_default.json 2> gpurun_out/${TAG}_default.err || exit $?
echo "default bench wall $(( $(date +%s) - s )) s"
timeout -k 10 200 python bench.py --vacuum --no-extra --no-cpu > gpurun_out/${TAG}_vac.json || exit $?
MNL_TILE=0 timeout -k 10 200 python bench.py --vacuum --no-extra --no-cpu > gpurun_out/${TAG}_vac_old.json || exit $?
MNL_TILE=0 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_wg_old.json || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r03b_*.json")):
    try: d=json.load(open(f))
    except Exception as e: print(f, e); continue
    r=d["roofline"]; g=r.get("general_kernel",{})
    print(f, d["value"], d["ms_per_step"], d["config"]["model_fraction_of_peak"], r["kernel"][:40], r["avg_launch_ms"], r["frac"], g.get("avg_launch_ms"))
    for k,v in (d.get("configs") or {}).items():
        print("   ", k, v.get("value"), v.get("ms_per_step"), v.get("model_fraction_of_peak"), v.get("roofline",{}).get("avg_launch_ms"))
PY
find gpurun_out/prof_${TAG} -name "*kernel_stats*"
