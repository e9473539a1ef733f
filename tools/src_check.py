import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from scenarios import ProductSim, make_oracle, vol
for comp in (0, 1, 2):
    res = []
    for make in (ProductSim, make_oracle):
        o = vol(make, 3, [3.2, 3.2, 3.2], 10, center_origin=True)
        o.add_gaussian_source(comp, 0.35, 4.0, 0.0, 40.0, (0.05, 0.05, 0.05), 25.0)
        o.step(1)
        res.append([o.get_array(c) for c in range(12)])
    for c in range(12):
        d = np.abs(res[0][c] - res[1][c])
        if d.max() > 0:
            w = np.argwhere(d > 0)[:2]
            print("src", comp, "comp", c, [(tuple(int(v) for v in ww), repr(res[0][c][tuple(ww)]), repr(res[1][c][tuple(ww)])) for ww in w])
        nz = np.argwhere(res[1][c] != 0)
        if c in (6, 7, 8) and len(nz):
            print("src", comp, "D comp", c, "nonzero pts", len(nz), [repr(res[1][c][tuple(ww)]) for ww in nz[:4]])
