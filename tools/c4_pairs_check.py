"""C4 (256^3 Kerr + Lorentzian slab) with and without pairs around the polarization chunks:
per-step time and the per-launch-family breakdown (HIP events).  Diagnostics for DESIGN.md
section 27."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402
from meep_nl_amd import core  # noqa: E402

core.set_verbosity(0)
wl = sys.argv[1] if len(sys.argv) > 1 else "kerr"
gv, s, f = bench.build_fields(wl, 256, 0, 1, 0, None)
if "--tune" in sys.argv:
    print("tuned", f.tune(), flush=True)
f.step(6)
print("tb_info", f.tb_info(), flush=True)
f.set_profiling(True)
names = {0: "tile", 2: "general", 5: "pair", 6: "rim", 4: "E"}
for v in (0, 1, 0, 1):
    f.set_schedule("tb_pol", v)
    f.step(4)
    base = {k: f.kernel_stats(k) for k in names}
    t0 = time.perf_counter()
    f.step(40)
    el = time.perf_counter() - t0
    parts = []
    for k, nm in names.items():
        n, ms, _ = f.kernel_stats(k)
        parts.append(f"{nm} {n - base[k][0]}x {(ms - base[k][1]) / 40:.4f}")
    print(f"tb_pol {v}: {el / 40 * 1e3:.4f} ms/step, active {f.tb_info()['active']}; per step: "
          + ", ".join(parts), flush=True)
