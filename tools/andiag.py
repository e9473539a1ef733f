"""Diagnostic: first step where the anisotropic-Lorentzian GPU run departs from the oracle."""
import sys; sys.path[:0] = ['tests', '.']
import numpy as np
from scenarios import ProductSim, make_oracle, sc_aniso_lorentz_3d
full = len(sys.argv) > 1
p = sc_aniso_lorentz_3d(ProductSim, steps=0, full=full)
o = sc_aniso_lorentz_3d(make_oracle, steps=0, full=full)
sh = p.shape()
for st in range(1, 41):
    p.step(1)
    o.step(1)
    bad = False
    for c in range(12):
        a, b = p.get_array(c), o.get_array(c)
        d = np.abs(a - b).reshape(sh)
        if d.max() > 0:
            idx = np.argwhere(d > 0)
            print("step", st, "comp", c, "ndiff", len(idx), "max", d.max(), "first", idx[:8].tolist(),
                  "vals", [(float(a.reshape(sh)[tuple(i)]), float(b.reshape(sh)[tuple(i)])) for i in idx[:3]])
            bad = True
    if bad:
        print("shape", sh)
        break
print("done", flush=True)
