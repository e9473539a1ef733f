"""One-rank fixtures of the multi-GPU self-check (bench.py c5_parity).

For each (S, N): the C5 grid of N slabs (S x S x N*S/4 cells, vacuum + PML(1.0), the Ez Gaussian
current at the centre) stepped on ONE GPU from the seeded random fields of
tests/scenarios.sc_c5_full (1 + 6 steps), its per-plane checksums of all twelve components
written to tests/golden/c5_parity_<grid>.npz.  A multi-rank bench run steps the same grid over
its ranks and compares the rank sums of its checksums with these, plane by plane.  The one-rank
run itself is pinned to the multi-rank product and the oracle's decomposition by
tests/test_gpu_mp.py::test_c5_full_size_chunk_invariance (8 IPC ranks vs one rank, bitwise).

  python tools/make_c5_fixture.py 512:2 512:4 512:8 256:2
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from meep_nl_amd import core
    core.set_verbosity(0)
    for spec in sys.argv[1:]:
        size, slabs = (int(x) for x in spec.split(":"))
        t0 = time.perf_counter()
        gv, cs, facts = bench.c5_parity_run(size, slabs, 0, 1, 0, None,
                                            log=lambda m: print(f"  {spec}: {m}", flush=True))
        n = list(gv.n)
        path = bench.c5_fixture_path(n)
        np.savez_compressed(path, checksums=cs, grid=np.array(n), steps=np.array([bench.C5_STEPS]),
                            t=np.array([facts["t"]]),
                            temporal_blocking=np.array([facts["temporal_blocking"]]))
        print(f"{spec}: grid {n}, t {facts['t']}, pairs {facts['temporal_blocking']}, "
              f"{time.perf_counter() - t0:.1f} s -> {os.path.relpath(path, ROOT)}", flush=True)


if __name__ == "__main__":
    main()
