import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from scenarios import ProductSim, make_oracle, sc_upstream_nl_3d
kw = dict(isrc=False, lorentz=False, chi2=False, pml=False)
for steps in (1, 2, 3, 5, 12):
    p = sc_upstream_nl_3d(ProductSim, steps=steps, **kw)
    o = sc_upstream_nl_3d(make_oracle, steps=steps, **kw)
    print(steps, "maxdiff per comp", [float(np.abs(p.get_array(c) - o.get_array(c)).max()) for c in range(12)])
p = sc_upstream_nl_3d(ProductSim, steps=12, **kw)
E = [p.get_array(c) for c in range(3)]; D = [p.get_array(6 + c) for c in range(3)]
chi3 = []; u = []
for c in range(3):
    x, y, z = p.coords(c); inside = np.abs(z - 0.2) < 0.9
    chi3.append(np.where(inside, 2e-2, 0.0)); u.append(np.where(inside, 1 / 2.25, 1.0))
def calc(Dsq, Di, ui, c2, c3v):
    cc2 = Di * c2 * (ui * ui); cc3 = Dsq * c3v * (ui * ui * ui)
    return (1 + cc2 + 2 * cc3) / (1 + 2 * cc2 + 3 * cc3)
for d in range(3):
    d1, d2 = (d + 1) % 3, (d + 2) % 3
    def nsum(e):
        g = D[e]
        return g + np.roll(g, -1, d) + np.roll(g, 1, e) + np.roll(np.roll(g, -1, d), 1, e)
    g1s = nsum(d1); g2s = nsum(d2); gs = D[d]
    dsq = gs * gs + 0.0625 * (g1s * g1s + g2s * g2s)
    Ep = (gs * u[d]) * calc(dsq, gs, u[d], 0.0, chi3[d])
    sl = tuple(slice(2, -2) for _ in range(3))
    diff = np.abs(Ep[sl] - E[d][sl])
    idx = np.unravel_index(np.argmax(diff), diff.shape)
    print("product E vs formula", d, diff.max(), np.count_nonzero(diff), idx)
