import sys, os, itertools
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from scenarios import ProductSim, make_oracle, vol
for f, w, et in itertools.product((0.15, 0.35), (10.0, 4.0), (100.0, 40.0)):
    res = []
    for make in (ProductSim, make_oracle):
        o = vol(make, 3, [1.6, 1.6, 1.6], 10, center_origin=True)
        o.add_gaussian_source(2, f, w, 0.0, et, (0.05, 0.05, 0.05), 1.0)
        vals = []
        for k in range(6):
            o.step(1)
            vals.append(o.get_array(8).copy())
        res.append(vals)
    print(f, w, et, [float(np.abs(a - b).max()) for a, b in zip(*res)])
