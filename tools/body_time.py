"""Tile-kernel time of one body class (diagnostics; masked runs are not valid fields):
MNL_TILE_BODY_MASK=<mask> [MNL_LIB_VARIANT=<lib>] python tools/body_time.py [--vacuum] [--size S]
Prints the tile kernel's HIP-event ms per launch (median of 5 batches of 10 steps)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

wl = "vacuum" if "--vacuum" in sys.argv else "waveguide"
size = int(sys.argv[sys.argv.index("--size") + 1]) if "--size" in sys.argv else 512
gv, s, f = bench.build_fields(wl, size, 0, 1, 0, None)
f.step(5)
res = []
for _ in range(5):
    f.set_profiling(True)
    f.step(10)
    n, ms, _ = f.kernel_stats(0)
    res.append(ms / max(n, 1))
res.sort()
print(f"mask {os.environ.get('MNL_TILE_BODY_MASK')} lib {os.environ.get('MNL_LIB_VARIANT', 'prod')}: "
      f"tile kernel {res[2]:.4f} ms (min {res[0]:.4f})", flush=True)
