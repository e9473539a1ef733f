"""Multi-rank overhead proxy on one GPU (diagnostics): the 512 x 512 x (P*W) vacuum + PML
grid stepped as one rank vs as W in-process z-slabs of P planes (LocalHub: one host thread
per slab, device-copy exchange, the ranks' kernels sharing the GPU).  Same total work per
step for W = 1 and the W-slab group of the same grid, so the ratio of their throughputs
bounds what the multi-rank step (chunk-0 launch, shell planes, exchanges) costs.
  python tools/local_scaling.py [P] [W ...]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from meep_nl_amd import core  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
WS = [int(v) for v in sys.argv[2:]] or [2, 4]


def run(total_planes, W, steps=20):
    n = [512, 512, total_planes]
    io = [-(v - (v & 1)) for v in n]
    gv = core.GridVolume(3, n, 10.0, io)
    s = core.Structure(gv, 0.5)
    s.add_pml(1.0)
    hub = core.LocalHub(W) if W > 1 else None
    fs = [core.Fields(s, rank=r, nranks=W, hub=hub) if W > 1 else core.Fields(s) for r in range(W)]
    for f in fs:
        f.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0, is_integrated=False)

    def par(fn):
        th = [threading.Thread(target=fn, args=(f,)) for f in fs]
        for t in th:
            t.start()
        for t in th:
            t.join()
    par(lambda f: f.step(8))
    t0 = time.perf_counter()
    par(lambda f: f.step(steps))
    el = time.perf_counter() - t0
    cells = 512.0 * 512.0 * total_planes
    fused = all(f.fused_active() for f in fs)
    del fs, hub, s
    return cells * steps / el / 1e9, el / steps * 1e3, fused


for W in WS:
    g1, ms1, f1 = run(P * W, 1)
    gW, msW, fW = run(P * W, W)
    print(f"grid 512x512x{P * W}: 1 rank {g1:.2f} G cells*steps/s ({ms1:.3f} ms/step, fused {f1}); "
          f"{W} slabs {gW:.2f} G ({msW:.3f} ms/step, fused {fW}); ratio {gW / g1:.3f}", flush=True)
