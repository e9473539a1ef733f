#!/bin/bash
# A/B of library variants on the GPU box: for each variant (base = the default
# libmnl.so) a short parity subset, then the 512^3 bench; one summary line each.
#   tools/ab_runs.sh base gw4 ...      (BENCH_ARGS / PARITY_K override the defaults)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
BARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu --no-extra}
PK=${PARITY_K:-"fused_big_box or fused_many_tiles or random_big_box or c2_256_random"}
for v in "$@"; do
  if [ "$v" = base ]; then unset MNL_LIB_VARIANT; else export MNL_LIB_VARIANT=$v; fi
  if [ -n "$PK" ] && [ "$PK" != none ]; then
    timeout -k 10 600 python -m pytest -x -q --timeout 500 --timeout-method thread -m gpu \
      tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_init.py tests/test_gpu_fullsize.py \
      -k "$PK" > gpurun_out/ab_parity_$v.log 2>&1
    rc=$?
    echo "== $v parity rc=$rc: $(tail -1 gpurun_out/ab_parity_$v.log)"
    [ $rc -ne 0 ] && exit $rc
  fi
  for rep in 1 2; do
    timeout -k 10 300 python bench.py $BARGS > gpurun_out/ab_bench_${v}_$rep.log 2>&1 || exit $?
    python - "$v" gpurun_out/ab_bench_${v}_$rep.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
g = r.get("general_kernel", {})
print(f"== {sys.argv[1]}: {d['ms_per_step']:.4f} ms/step  lean {r['avg_launch_ms']:.4f}  general {g.get('avg_launch_ms', 0):.4f}  value {d['value']}")
PY
  done
done
