"""Start-up cost of the 512^3 bench workload (diagnostics): structure + fields creation,
then the first steps one call at a time (the first step runs unfused; the second enters
the fused mode: geometry, palette, ping-pong buffers)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 512
t0 = time.perf_counter()
gv, s, f = bench.build_fields("waveguide", size, 0, 1, 0, None)
print(f"build_fields {time.perf_counter() - t0:.3f} s", flush=True)
for i in range(4):
    t0 = time.perf_counter()
    f.step(1)
    print(f"step {i + 1}: {time.perf_counter() - t0:.3f} s (fused {f.fused_active()})", flush=True)
