"""Structure dump / load (structure::dump / load, src/structure_dump.cpp) is
host-only: round trip, grid mismatch and corruption errors (no GPU needed).
The fields half (mnl_fields_dump / load) is covered on the GPU by
tests/test_gpu_checkpoint.py."""
import numpy as np
import pytest

from meep_nl_amd import core


def _structure():
    gv = core.GridVolume.vol(3, [1.6, 1.2, 1.4], 10, center_origin=True)
    s = core.Structure(gv)
    s.add_pml(0.4)
    x, y, z = gv.coords(0)
    s.set_chi1inv(0, 0, np.where(np.abs(y) < 0.3, 0.25, 1.0))
    s.set_chi2(1, np.full(gv.shape(), 0.1))
    s.set_conductivity(6, np.where(x < 0, 0.5, 0.0))
    s.add_lorentzian(1.1, 0.05, [np.full(gv.shape(), 0.5), None, None])
    s.set_box(0, [-0.2, 0.2, -0.2, 0.2, -0.2, 0.2], 3.0)
    return gv, s


def test_structure_roundtrip(tmp_path):
    gv, s = _structure()
    p1, p2 = str(tmp_path / "a.mnl"), str(tmp_path / "b.mnl")
    s.dump(p1)
    t = core.Structure(gv)
    t.load(p1)
    t.dump(p2)
    assert open(p1, "rb").read() == open(p2, "rb").read()


def test_structure_load_errors(tmp_path):
    gv, s = _structure()
    p = str(tmp_path / "a.mnl")
    s.dump(p)
    other = core.Structure(core.GridVolume.vol(3, [1.6, 1.2, 1.6], 10, center_origin=True))
    with pytest.raises(RuntimeError, match="different grid volume"):
        other.load(p)
    data = open(p, "rb").read()
    open(p, "wb").write(data[:-9])
    with pytest.raises(RuntimeError, match="truncated or corrupt"):
        core.Structure(gv).load(p)
    open(p, "wb").write(b"garbage!" + data[8:])
    with pytest.raises(RuntimeError, match="not a structure file"):
        core.Structure(gv).load(p)
