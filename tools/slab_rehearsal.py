#!/usr/bin/env python3
"""Rehearsal of the multi-GPU decomposition on ONE GPU: the 512x512x512 waveguide
as 1 slab, then as P in-process z-slabs (mnl_fields_create_local: the same
decomposition, fused multi-rank step and halo exchange code as the RCCL path,
with device copies instead of xGMI).  All slabs share one GPU, so the ideal is
the same cells*steps/s as the single slab; the gap is the overhead of the
multi-rank step (split kernels, chunk 0 on the side stream, top-plane shell
kernels, exchanges) that each GPU pays at N > 1.
  python tools/slab_rehearsal.py [--weak] [P ...]
--weak: every slab keeps a full 512^3 (global 512x512x512P, as bench.py --gpus P);
the ideal is then P times the single-slab step time."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from meep_nl_amd import core  # noqa: E402


WEAK = "--weak" in sys.argv


def build(nr, hub=None, rank=0):
    n = [512, 512, 512 * (nr if WEAK else 1)]
    io = [-v for v in n]
    gv = core.GridVolume(3, n, 10.0, io)
    s = core.Structure(gv, 0.5)
    s.add_pml(1.0)
    big = 1e9
    s.set_box(0, [-big, big, -0.5 + 1e-12, 0.5 - 1e-12, -0.5 + 1e-12, 0.5 - 1e-12], 12.0)
    return gv, s


def run(P, steps=40, warm=6):
    gv, s = build(P)
    if P == 1:
        fs = [core.Fields(s)]
    else:
        hub = core.LocalHub(P)
        fs = [core.Fields(s, rank=r, nranks=P, hub=hub) for r in range(P)]
    for f in fs:
        f.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)

    def par(n):
        th = [threading.Thread(target=lambda f=f: f.step(n)) for f in fs]
        for t in th:
            t.start()
        for t in th:
            t.join()
    par(warm)
    t0 = time.perf_counter()
    par(steps)
    el = time.perf_counter() - t0
    fused = all(f.fused_active() for f in fs)
    cells = 512.0 ** 3 * (P if WEAK else 1)
    print(f"slabs {P}: {el / steps * 1e3:.3f} ms/step, {cells * steps / el / 1e6:.0f} Mcells*steps/s,"
          f" fused={fused}", flush=True)
    del fs


if __name__ == "__main__":
    for P in [int(a) for a in sys.argv[1:] if a != "--weak"] or [1, 2, 4]:
        run(P)
