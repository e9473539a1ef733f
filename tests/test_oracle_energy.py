"""Field energy (fields::field_energy / electric_energy_in_box /
magnetic_energy_in_box, src/energy_and_flux.cpp:48-178) in the CPU oracle,
pinned to the reference's own tests.

The reference's C++ tests run complex fields (no use_real_fields()), and the
energy integrand real(conj(E) D) adds the real and imaginary parts' energies.
The whole update is linear with real coefficients, so the imaginary part is
the real-field run driven by amplitude -i*A: energy(complex run, A) =
energy(real run, A) + energy(real run, -i*A)."""
import math

import numpy as np
import pytest

import scenarios as S
from scenarios import make_oracle


def polariton_energy(make, amp):
    o = S.vol(make, 1, [1], 10)
    o.add_lorentzian(0.3, 0.1, [np.full(o.shape(), 7.63), None, None])
    o.legacy_point_source(0, 0.2, 3.0, 0.0, 2.0, o.center(), amp)
    n = 0
    while float(np.float32(n * (0.5 / 10))) < 10.0:
        n += 1
    o.step(n)
    return o.field_energy()


def test_polariton_energy_golden(golden):
    """tests/known_results.cpp:156: 1-D polariton energy 0.0863443 (rel 1e-5)."""
    A = complex(0, -2 * math.pi * 0.2)
    e = polariton_energy(make_oracle, A) + polariton_energy(make_oracle, -1j * A)
    ref = golden["known_results"]["polariton_energy_1d"]
    assert abs(e - ref) <= abs(ref) * 1e-5, e


def pml_energies(make, amp):
    o = make(3, [15, 10, 12], 10.0, 0.5, [0, 0, 0])
    o.add_pml(0.401)
    o.legacy_point_source(2, 0.8, 0.6, 0.0, 4.0, (0.751, 0.5, 0.601), amp)
    ts = S.legacy_last_time(0.8, 0.6, 0.0, 4.0, 10.0, 0.05)
    while o.time() < ts:
        o.step()
    out, check = [o.field_energy()], 10.0
    while o.time() < 31.0:
        o.step()
        if o.time() >= check:
            out.append(o.field_energy())
            check += 10.0
    return out


def test_three_d_pml_energy_decay():
    """tests/three_d.cpp:163-194 (test_pml): after the source, the field energy
    falls below 4e-3 of its end-of-source value within 10 time units, and stays
    there at 20 and 30."""
    a = pml_energies(make_oracle, 1.0)
    b = pml_energies(make_oracle, -1j)
    e = [x + y for x, y in zip(a, b)]
    assert len(e) == 4 and e[0] > 0
    for v in e[1:]:
        assert v <= e[0] * 4e-3, (v, e[0])


def test_energy_trapezoid_and_parts():
    """Electric energy over a box whose faces lie on Ex grid points is the
    trapezoid rule of Ex.Dx/2 (weight 1/2 on the faces, loop_in_chunks
    boundary weights); field_energy = electric + synchronized magnetic, and the
    synchronization leaves every field array as it was."""
    o = S.vol(make_oracle, 3, [1.6, 1.4, 1.2], 10, center_origin=True)
    o.add_pml(0.4)
    S.random_init(o, (6,))  # Dx only: Ey = Ez = 0, E from D through update_eh
    lo, hi = [-0.35, -0.3, -0.2], [0.25, 0.2, 0.4]
    ex, dx = o.get_array(0), o.get_array(6)
    x, y, z = o.coords(0)
    w = np.ones(ex.shape)
    for v, l, h in ((x, lo[0], hi[0]), (y, lo[1], hi[1]), (z, lo[2], hi[2])):
        inside = (v > l - 1e-9) & (v < h + 1e-9)
        edge = np.isclose(v, l) | np.isclose(v, h)
        w = w * np.where(inside, np.where(edge, 0.5, 1.0), 0.0)
    want = 0.5 * np.sum(w * ex * dx) * 1e-3
    got = o.electric_energy_in_box(lo, hi)
    assert got == pytest.approx(want, rel=1e-13)
    S.random_init(o, (9, 10, 11, 7, 8), seed=3)
    o.step(3)
    before = [o.get_array(c).copy() for c in range(12)]
    el, mag = o.electric_energy_in_box(), o.magnetic_energy_in_box()
    tot = o.field_energy()
    for c in range(12):
        np.testing.assert_array_equal(o.get_array(c), before[c])
    assert o.electric_energy_in_box() == el and o.magnetic_energy_in_box() == mag
    assert tot != el + mag and tot > 0
