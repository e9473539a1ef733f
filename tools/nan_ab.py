"""In-process A/B of the device NaN guard: the bench workload (512^3
waveguide), tuned, then alternating segments of --seg steps with the guard every step and
with it thinned to never; prints ms/step per segment and the medians.  One process, one set of
allocations: the box-to-box and process-to-process spread (page placement) cancels.
  python tools/nan_ab.py [--size 512] [--seg 100] [--reps 4]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--seg", type=int, default=100)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    import bench
    gv, s, f = bench.build_fields("waveguide", a.size, 0, 1, 0, None)
    f.tune()
    f.step(10)
    res = {1: [], 10 ** 9: []}
    for r in range(a.reps):
        for every in (1, 10 ** 9):
            f.set_nan_check(every)
            t0 = time.perf_counter()
            f.step(a.seg)
            ms = (time.perf_counter() - t0) / a.seg * 1e3
            res[every].append(ms)
            print(f"rep {r} guard {'every step' if every == 1 else 'never'}: {ms:.4f} ms/step",
                  flush=True)
    on, off = statistics.median(res[1]), statistics.median(res[10 ** 9])
    print(f"median: guard every step {on:.4f}, never {off:.4f} ms/step, overhead "
          f"{(on / off - 1) * 100:.2f} %")


if __name__ == "__main__":
    main()
