#!/bin/bash
# C4-NR (256^3) per-variant step time and E-update time: tools/nr_ab.sh base prev ...
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
for v in "$@"; do
  if [ "$v" = base ]; then unset MNL_LIB_VARIANT; else export MNL_LIB_VARIANT=$v; fi
  timeout -k 10 300 python - "$v" <<'PY' || exit $?
import sys, time
sys.path.insert(0, ".")
import bench
gv, s, f = bench.build_fields("kerr_nr", 256, 0, 1, 0, None)
f.step(5)
f.set_profiling(True)
t0 = time.perf_counter(); f.step(20); el = time.perf_counter() - t0
n, ms, _ = f.kernel_stats(4)
print(f"== {sys.argv[1]}: {el / 20 * 1e3:.4f} ms/step, E update {ms / max(n, 1):.4f} ms, timers {f.timers()}")
PY
done
