#!/bin/bash
# Bench the 512^3 headline under different environment settings, one summary
# line per run (timing experiments; no parity):
#   tools/env_runs.sh "" "MNL_EXPT=1" "MNL_FUSED_ZCHUNK=16 MNL_EXPT=2"
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
BARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu --no-extra}
REPS=${REPS:-2}
i=0
for spec in "$@"; do
  i=$((i + 1))
  for rep in $(seq $REPS); do
    log=gpurun_out/env_${i}_$rep.log
    env $spec timeout -k 10 300 python bench.py $BARGS > $log 2>&1 || { echo "== [$spec] failed"; tail -5 $log; exit 1; }
    python - "$spec" $log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
g = r.get("general_kernel", {})
print(f"== [{sys.argv[1]}]: {d['ms_per_step']:.4f} ms/step  lean {r['avg_launch_ms']:.4f}  general {g.get('avg_launch_ms', 0):.4f}")
PY
  done
done
