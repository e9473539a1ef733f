"""The tuner's choices and per-candidate times on one workload (MNL_TUNE_VERBOSE), then the
stepped time of the tuned fields over a few repeats (diagnostics of the tuner, round 6)."""
import os
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
os.environ.setdefault("MNL_TUNE_VERBOSE", "1")
import bench  # noqa: E402
from meep_nl_amd import core  # noqa: E402

core.set_verbosity(0)
wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 256
gv, s, f = bench.build_fields(wl, size, 0, 1, 0, None)
print("tuned", f.tune(), f.tb_info(), flush=True)
f.step(6)
for r in range(4):
    t0 = time.perf_counter()
    f.step(40)
    print(f"repeat {r}: {(time.perf_counter() - t0) / 40 * 1e3:.4f} ms/step", flush=True)
