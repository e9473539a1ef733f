"""CPU checks of the oracle's DFT-fields restatement (fields::add_dft_fields,
src/dft.cpp:889-903; fields::get_dft_array / process_dft_component / collapse_array,
src/dft.cpp:908-1280, src/array_slice.cpp:525-601).

Parity pin: the fork holds no golden DFT-field values (tests/dft-fields.cpp
compares against solve_cw + HDF5, python/tests/test_dft_fields.py against HDF5
output).  The restatement is pinned instead by
  * an independent numpy time-domain DFT of the oracle's own Yee arrays (the
    definition the reference accumulates: sum_t f(t) e^{i w t} dt/sqrt(2 pi), t the
    E time or t - dt/2 for H, src/dft.cpp:249-300) on the Yee grid and, averaged
    onto cell centres, on the centered grid (rel 1e-12);
  * python/tests/test_dft_fields.py's properties: thin volumes collapse to 1-D
    arrays, a flux object's array equals the fields object's on the same plane,
    decimated DFT fields agree with undecimated ones to 1e-3.
"""
import math

import numpy as np
import pytest

from scenarios import make_oracle, vol

FR = [0.25, 0.3]


def _run(steps=300, decim=1):
    o = vol(make_oracle, 2, [4, 4], 10)
    o.add_pml(1.0)
    o.add_gaussian_source(2, 0.3, 5.0, 0.0, 50.0, (0.3, 0.2, 0), 1.0)
    hs = {
        "cent": o.add_dft_fields([2, 3], [0, 0, 0], [4, 4, 0], FR, False, decim),
        "yee": o.add_dft_fields([2, 4], [0, 0, 0], [4, 4, 0], FR, True, decim),
        "thin_x": o.add_dft_fields([2], [1.5, 0.5, 0], [1.5, 3.5, 0], FR, False, decim),
        "flux_x": o.add_dft_flux([([1.5, 0.5, 0], [1.5, 3.5, 0], 0, 1.0)], FR, decim),
        "thin_y": o.add_dft_flux([([0.0, 1.0, 0], [4.0, 1.0, 0], 1, 1.0)], FR, decim),
    }
    return o, hs


def test_dft_fields_equal_numpy_dft():
    o, hs = _run(steps=0)
    acc_e = np.zeros((len(FR),) + o.shape(), complex)
    acc_h = np.zeros((len(FR),) + o.shape(), complex)
    dt = o.dt
    for _ in range(300):
        o.step(1)
        t = o.t * dt
        ez, hy = o.get_array(2), o.get_array(4)
        for i, f in enumerate(FR):
            acc_e[i] += ez * np.exp(1j * 2 * math.pi * f * t) * dt / math.sqrt(2 * math.pi)
            acc_h[i] += hy * np.exp(1j * 2 * math.pi * f * (t - 0.5 * dt)) * dt / math.sqrt(2 * math.pi)
    for i in range(len(FR)):
        # Yee grid: Ez (unshifted in x, y) owned points 1..n; Hy (x shifted) 0..n-1, y 1..n
        ez = o.dft_array(hs["yee"], 2, i)
        assert ez.shape == (40, 40)
        ref = acc_e[i][1:41, 1:41]
        assert np.max(np.abs(ez - ref)) <= 1e-12 * np.max(np.abs(ref))
        hy = o.dft_array(hs["yee"], 4, i)
        ref = acc_h[i][0:40, 1:41]
        assert np.max(np.abs(hy - ref)) <= 1e-12 * np.max(np.abs(ref))
        # centered grid: cell centres (2 i + 1), the 4-point average of Ez's Yee values
        ec = o.dft_array(hs["cent"], 2, i)
        a = acc_e[i]
        ref = 0.25 * (a[0:40, 0:40] + a[1:41, 0:40] + a[0:40, 1:41] + a[1:41, 1:41])
        assert ec.shape == (40, 40)
        assert np.max(np.abs(ec - ref)) <= 1e-12 * np.max(np.abs(ref))


def test_collapse_and_flux_array():
    """python/tests/test_dft_fields.py::test_get_dft_array: thin volumes give 1-D
    arrays; a flux plane's array equals the fields object's on the same plane."""
    o, hs = _run()
    o.step(300)
    tx, fx = o.dft_array(hs["thin_x"], 2, 0), o.dft_array(hs["flux_x"], 2, 0)
    ty = o.dft_array(hs["thin_y"], 2, 0)
    assert tx.ndim == 1 and ty.ndim == 1 and tx.shape == (32,) and ty.shape == (40,)
    assert np.max(np.abs(tx - fx)) <= 1e-13 * np.max(np.abs(tx))
    assert np.any(tx != 0) and np.any(ty != 0)
    with pytest.raises(RuntimeError, match="outside the range"):
        o.dft_array(hs["cent"], 2, 2)
    assert o.dft_array(hs["cent"], 0, 0).size == 0  # no Ex chunks: rank 0, no array


def test_decimated_close_to_undecimated():
    """python/tests/test_dft_fields.py: decimation_factor=4 vs 1 within 1e-3."""
    o, hs = _run()
    h4 = o.add_dft_fields([2], [0, 0, 0], [4, 4, 0], FR, False, 4)
    o.step(4000)  # until the pulse (width 5, cutoff 5 widths) has left through the PML
    a1, a4 = o.dft_array(hs["cent"], 2, 0), o.dft_array(h4, 2, 0)
    assert np.linalg.norm(a1 - a4) <= 1e-3 * np.linalg.norm(a1)
