#!/usr/bin/env python3
"""Diagnostics: step time of the bench workload in several timed segments of one
process (is run-to-run variance within a process or between processes?)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sys.argv = [sys.argv[0], "--no-cpu"] + sys.argv[1:]
args = bench.parse()
if args.workload is None:
    args.workload = "vacuum" if args.vacuum else "waveguide"
gv, s, f = bench.build_fields(args, 0, 1, 0, None)
f.step(10)
out = []
for seg in range(6):
    t0 = time.perf_counter()
    f.step(30)
    out.append((time.perf_counter() - t0) / 30 * 1e3)
print("segments ms/step:", " ".join(f"{v:.3f}" for v in out), "alloc", f.alloc_info())
