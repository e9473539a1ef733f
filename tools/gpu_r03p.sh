#!/bin/bash
# Round-3 final measurements with the tuner: the default bench as the driver runs it (wall
# time recorded), the vacuum headline, C5 at N=1; rocprof kernel stats + PMC passes of the
# 512^3 waveguide and vacuum tile kernel at the z-chunk each bench kept (--no-tune with
# MNL_FUSED_ZCHUNK set, so every profiled launch is the timed region's configuration).
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
s=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/r03p_default.json 2> gpurun_out/r03p_default.err || exit $?
echo "default bench wall $(( $(date +%s) - s )) s" | tee gpurun_out/r03p_wall.txt
timeout -k 10 200 python bench.py --vacuum --no-extra --no-cpu > gpurun_out/r03p_vac.json || exit $?
timeout -k 10 200 python bench.py --workload c5 --no-extra --no-cpu > gpurun_out/r03p_c5.json || exit $?
zc() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(max(d['config']['tuned_zchunk_gen_cus'][0], 0))" $1; }
ZW=$(zc gpurun_out/r03p_default.json); ZV=$(zc gpurun_out/r03p_vac.json)
echo "zchunk waveguide $ZW vacuum $ZV"
MNL_FUSED_ZCHUNK=$ZW TAG=r03p_wg BENCH_ARGS="--steps 10 --warmup 2 --no-cpu --no-extra --no-tune" bash tools/gpu_pmc.sh || exit $?
MNL_FUSED_ZCHUNK=$ZV TAG=r03p_vac BENCH_ARGS="--vacuum --steps 10 --warmup 2 --no-cpu --no-extra --no-tune" bash tools/gpu_pmc.sh || exit $?
python - <<'PY'
import json
for f in ("r03p_default", "r03p_vac", "r03p_c5"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], d["config"]["model_fraction_of_peak"], r["avg_launch_ms"], r["frac"],
          d["config"].get("tuned_zchunk_gen_cus"))
    for k, v in (d.get("configs") or {}).items():
        print("   ", k, v.get("value"), v.get("ms_per_step"), v.get("model_fraction_of_peak"), v.get("tuned_zchunk_gen_cus"))
PY
