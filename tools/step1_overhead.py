"""Host overhead of one-step calls (diagnostics): the 512^3 bench workload stepped as
step(50) and as 50 x step(1); prints ms/step for both."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

wl = "vacuum" if "--vacuum" in sys.argv else "waveguide"
size = int(sys.argv[sys.argv.index("--size") + 1]) if "--size" in sys.argv else 512
gv, s, f = bench.build_fields(wl, size, 0, 1, 0, None)
f.step(10)
for rep in range(2):
    t0 = time.perf_counter()
    f.step(50)
    a = (time.perf_counter() - t0) / 50 * 1e3
    t0 = time.perf_counter()
    for _ in range(50):
        f.step(1)
    b = (time.perf_counter() - t0) / 50 * 1e3
    print(f"{wl} {size}^3: step(50) {a:.3f} ms/step, step(1) x 50 {b:.3f} ms/step", flush=True)
