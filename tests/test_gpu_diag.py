"""Diagnostics builds of the persistent kernels (MNL_ITEM_CLOCK, tools/item_clock.py): the
per-item records are written, every item of every launch is recorded once, and the fields
are bitwise those of the normal kernels (the clock only reads a counter and stores records)."""
import os

import numpy as np
import pytest

from scenarios import ProductSim, sc_waveguide_3d

pytestmark = pytest.mark.gpu


def _records(path):
    raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    out, i = [], 0
    while i < len(raw):
        assert int(raw[i, 0]) == 0x4b4c434d4e4d
        n = int(raw[i, 2])
        out.append(raw[i + 1:i + 1 + n])
        i += 1 + n
    return np.concatenate(out) if out else np.zeros((0, 8), np.uint64)


@pytest.mark.parametrize("tb", ["1", "0"])
def test_item_clock_records_and_bitwise(tmp_path, monkeypatch, tb):
    monkeypatch.setenv("MNL_TB", tb)
    ref = sc_waveguide_3d(ProductSim, L=6.4, steps=12)
    assert ref._fields().fused_active()
    want = {c: ref.get_array(c) for c in range(12)}
    del ref
    path = str(tmp_path / "clk.bin")
    monkeypatch.setenv("MNL_ITEM_CLOCK", path)
    p = sc_waveguide_3d(ProductSim, L=6.4, steps=12)
    for c in range(12):
        assert p.get_array(c).tobytes() == want[c].tobytes(), c
    r = _records(path)
    assert len(r) > 0
    kinds = set(int(k) for k in (r[:, 2] & 0xFF))
    assert kinds <= {0, 1, 2}
    if tb == "1" and p._fields().tb_info()["active"]:
        assert {1, 2} <= kinds  # rim launches and two-step items of the pairs
    assert np.all(r[:, 1] >= r[:, 0])  # end after start
    os.unlink(path)
