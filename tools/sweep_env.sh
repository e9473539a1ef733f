#!/bin/bash
# Bench the 512^3 workload under several env settings: VARIANTS="A=1 B=2,C=3 ..."
# (comma joins several assignments in one variant).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-"X=0"}; do
  env $(echo $v | tr ',' ' ') timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu ${BENCH_EXTRA} > gpurun_out/sw.log 2>&1 || exit $?
  python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/sw.log").read().strip().splitlines()[-1])
r = d["roofline"]
g = r.get("general_kernel", {})
print(sys.argv[1], d["value"], d["ms_per_step"], "lean", r["avg_launch_ms"], "gen", g.get("avg_launch_ms"))
PY
done
