"""One masked tile-kernel run for PMC profiling (diagnostics; masked runs do not
produce valid fields): MNL_TILE_BODY_MASK=<mask> python tools/tile_one.py [--vacuum]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

wl = "vacuum" if "--vacuum" in sys.argv else "waveguide"
gv, s, f = bench.build_fields(wl, 512, 0, 1, 0, None)
f.step(3)
f.step(10)
print("ok", flush=True)
