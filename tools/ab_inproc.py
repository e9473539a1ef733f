#!/usr/bin/env python3
"""In-process A/B of env-selected kernel variants (same allocations, so physical
placement cannot bias the comparison):
  python tools/ab_inproc.py MNL_LEAN_GROUPS=1 MNL_LEAN_GROUPS=8 [-- bench args]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

argv = sys.argv[1:]
extra = argv[argv.index("--") + 1:] if "--" in argv else []
variants = argv[:argv.index("--")] if "--" in argv else argv
sys.argv = [sys.argv[0], "--no-cpu"] + extra
args = bench.parse()
if args.workload is None:
    args.workload = "vacuum" if args.vacuum else "waveguide"
gv, s, f = bench.build_fields(args.workload, args.size, 0, 1, 0, None)
f.step(10)
res = {v: [] for v in variants}
for rep in range(4):
    for v in variants:
        for kv in v.split(","):
            k, val = kv.split("=")
            os.environ[k] = val
        f.step(4)
        t0 = time.perf_counter()
        f.step(30)
        res[v].append((time.perf_counter() - t0) / 30 * 1e3)
for v in variants:
    print(v, "ms/step:", " ".join(f"{x:.3f}" for x in res[v]), "min", f"{min(res[v]):.3f}")
