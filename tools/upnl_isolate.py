import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from scenarios import ProductSim, make_oracle, compare_all, ALL_COMPS, sc_upstream_nl_3d
for kw in [dict(), dict(isrc=False), dict(lorentz=False), dict(chi2=False), dict(pml=False),
           dict(isrc=False, lorentz=False), dict(isrc=False, lorentz=False, chi2=False),
           dict(isrc=False, lorentz=False, chi2=False, pml=False)]:
    d = compare_all(sc_upstream_nl_3d(ProductSim, steps=20, **kw), sc_upstream_nl_3d(make_oracle, steps=20, **kw), ALL_COMPS)
    print(kw, max(d.values()), {c: v for c, v in d.items() if v})
