import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from scenarios import ProductSim, make_oracle, sc_upstream_nl_3d, vol
for kw in (dict(upstream=False, isrc=False, lorentz=False, chi2=False, pml=False),
           dict(upstream=False, isrc=False, lorentz=False, chi2=False, pml=False)):
    p = sc_upstream_nl_3d(ProductSim, steps=1, **kw)
    o = sc_upstream_nl_3d(make_oracle, steps=1, **kw)
    print(kw, [float(np.abs(p.get_array(c) - o.get_array(c)).max()) for c in range(12)])
# bare: only the Ey current source, vacuum
for amp, pos in ((25.0, (-0.4, 0.25, 0.35)), (1.0, (-0.4, 0.25, 0.35)), (25.0, (0.05, 0.05, 0.05))):
    res = []
    for make in (ProductSim, make_oracle):
        o = vol(make, 3, [3.2, 3.2, 3.2], 10, center_origin=True)
        o.add_gaussian_source(1, 0.35, 4.0, 0.0, 40.0, pos, amp)
        o.step(1)
        res.append(o.get_array(7))
    d = np.abs(res[0] - res[1])
    print("bare Ey src", amp, pos, float(d.max()), np.argwhere(d > 0)[:4].tolist(), res[0][d > 0][:3], res[1][d > 0][:3])
