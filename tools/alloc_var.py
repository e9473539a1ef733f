"""Spread of the headline step time over fresh allocations inside one process (DESIGN.md
section 7: between processes the same kernels vary with page placement).  Builds the 512^3
waveguide --allocs times with fixed knobs (no tuning), steps --steps after a warm-up each time.

  python tools/alloc_var.py [--allocs 5] [--steps 30] [--size 512]
"""
import argparse
import gc
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--allocs", type=int, default=5)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json")
    a = ap.parse_args()
    import bench
    from meep_nl_amd import core
    core.set_verbosity(0)
    out, parts = [], []
    for i in range(a.allocs):
        gv, s, f = bench.build_fields("waveguide", a.size, 0, 1, 0, None)
        f.step(8)
        f.set_profiling(True)
        ms = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            f.step(a.steps)
            ms.append((time.perf_counter() - t0) / a.steps * 1e3)
        out.append(min(ms))
        n5, ms5, _ = f.kernel_stats(5)  # pairs: all launches of a pair
        n6, ms6, _ = f.kernel_stats(6)  # rim launches that run alone
        parts.append({"pair_ms": ms5 / max(n5, 1), "rim_alone_ms": ms6 / max(n6, 1)})
        print(f"allocation {i}: {min(ms):.4f} ms/step (reps {[round(x, 4) for x in ms]}) "
              f"{parts[-1]}", flush=True)
        del f, s, gv
        gc.collect()
    res = {"size": a.size, "steps": a.steps, "ms_per_step": out, "parts": parts,
           "min": min(out), "max": max(out),
           "median": statistics.median(out), "env": {k: v for k, v in os.environ.items() if k.startswith("MNL_")}}
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
