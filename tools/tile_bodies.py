"""Per-body timing of the tile kernel (diagnostics; results of masked runs are NOT
valid fields): for each body mask, build the bench workload, step one-step (no temporal
blocking), and report the tile kernel's HIP-event time per launch.
python tools/tile_bodies.py [--workload waveguide|vacuum|c2|kerr|kerr_nr] [--size S]"""
import os
import sys
import time
import gc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    size = int(sys.argv[sys.argv.index("--size") + 1]) if "--size" in sys.argv else 512
    wl = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "waveguide"
    os.environ["MNL_TILE_STATS"] = "1"
    os.environ["MNL_TB"] = "0"
    for mask in (-1, 1, 2, 4, 8, 32, 64, 128, 254):
        os.environ["MNL_TILE_BODY_MASK"] = str(mask)
        gv, s, f = bench.build_fields(wl, size, 0, 1, 0, None)
        f.step(5)
        f.set_profiling(True)
        t0 = time.perf_counter()
        f.step(20)
        el = time.perf_counter() - t0
        n, ms, b = f.kernel_stats(0)
        g_n, g_ms, _ = f.kernel_stats(2)
        print(f"{wl} {size}^3 mask {mask:3d}: step {el / 20 * 1e3:.4f} ms, tile kernel "
              f"{ms / max(n, 1):.4f} ms, general kernel {g_ms / max(g_n, 1):.4f} ms", flush=True)
        del f, s
        gc.collect()


if __name__ == "__main__":
    main()
