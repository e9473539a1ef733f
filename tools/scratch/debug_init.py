import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import scenarios as S
for kw in [dict(steps=0), dict(steps=1), dict(steps=2), dict(steps=1, eps=12.0), dict(steps=2, eps=12.0), dict(steps=0, dpml=0.0), dict(steps=1, dpml=0.0), dict(steps=2, dpml=0.0)]:
    p = S.sc_random_fields(S.ProductSim, **kw)
    o = S.sc_random_fields(S.make_oracle, **kw)
    d = S.compare_all(p, o)
    bad = {c: v for c, v in d.items() if v}
    print(kw, "fused" if p._fields().fused_active() else "unfused", bad, flush=True)
    for c in bad:
        a, b = p.get_array(c), o.get_array(c)
        idx = np.argwhere(a != b)
        print("   comp", c, "n", len(idx), "first", idx[:4].tolist(), "shape", a.shape, flush=True)
