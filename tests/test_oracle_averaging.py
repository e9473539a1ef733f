"""Subpixel averaging in the oracle (structure::set_epsilon with anisotropic
averaging over a material function, src/anisotropic_averaging.cpp:33-298) and
the unit-sphere quadrature of src/sphere-quad.cpp, on the CPU.

Pinning: the reference's generated table (sphere-quad.h) is a build artefact
that is not in the reference tree, and running its generator here was refused
(DESIGN.md §22), so the quadrature restatements (product host code and oracle,
written independently) are checked against each other bit for bit and against
the defining properties of the formulas (unit points, weights, polynomial
exactness of the 50-point degree-11 and 12-point rules, the generator's
max-min-distance ordering).  eff_chi1inv_row is checked against the closed forms
it must reproduce: uniform media give the scalar 1/eps, a planar interface gives
the harmonic mean along its normal and the arithmetic mean across it (Kottke's
tensor), maxeval = 0 gives 1/eps at the pixel centre.
"""
import ctypes
import itertools
import math

import numpy as np
import pytest

import oracle.oracle as orc


def _double_factorial(n):
    return 1 if n <= 0 else n * _double_factorial(n - 2)


def _sphere_mean(a, b, c):
    """Mean of x^a y^b z^c over the unit sphere S^2."""
    if a % 2 or b % 2 or c % 2:
        return 0.0
    return (_double_factorial(a - 1) * _double_factorial(b - 1) * _double_factorial(c - 1) /
            _double_factorial(a + b + c + 1))


def test_quadrature_product_equals_oracle():
    from meep_nl_amd._lib import dptr, lib
    for dim in (1, 2, 3):
        n = lib().mnl_sphere_quadrature(dim, None)
        a = np.zeros((n, 4))
        lib().mnl_sphere_quadrature(dim, a.ctypes.data_as(dptr))
        b = orc.sphere_quadrature(dim)
        assert a.shape == b.shape == ({1: 2, 2: 12, 3: 50}[dim], 4)
        assert a.tobytes() == b.tobytes()


def test_quadrature_3d_is_degree_11():
    q = orc.sphere_quadrature(3)
    x, y, z, w = q.T
    assert np.allclose(x * x + y * y + z * z, 1.0, rtol=0, atol=1e-15)
    assert abs(w.sum() - 1.0) < 1e-15
    # McLaren's weights: 6 x 9216, 12 x 16384, 8 x 15309, 24 x 14641 (/725760)
    vals, counts = np.unique(np.round(w * 725760.0), return_counts=True)
    assert dict(zip(vals.astype(int), counts)) == {9216: 6, 14641: 24, 15309: 8, 16384: 12}
    for a, b, c in itertools.product(range(12), repeat=3):
        if a + b + c > 11:
            continue
        got = float(np.sum(w * x ** a * y ** b * z ** c))
        assert abs(got - _sphere_mean(a, b, c)) < 1e-14, (a, b, c)
    # degree 12 is not integrated exactly (the rule is degree 11)
    assert abs(float(np.sum(w * x ** 12)) - _sphere_mean(12, 0, 0)) > 1e-6


def test_quadrature_2d_and_1d():
    q = orc.sphere_quadrature(2)
    x, y, z, w = q.T
    assert np.all(z == 0) and np.all(w == 1.0 / 12)
    ang = np.sort(np.mod(np.arctan2(y, x), 2 * np.pi))
    assert np.allclose(np.diff(ang), 2 * np.pi / 12, atol=1e-14)
    for k in range(1, 12):  # trigonometric exactness below degree 12
        assert abs(np.sum(w * np.cos(k * np.arctan2(y, x)))) < 1e-14
    q1 = orc.sphere_quadrature(1)
    assert q1.tolist() == [[0, 0, 1, 0.5], [0, 0, -1, 0.5]]


@pytest.mark.parametrize("dim", [2, 3])
def test_quadrature_order_maximises_spacing(dim):
    """sort_by_distance: each point maximises its (single-precision) minimum squared
    distance to the points before it (ties: the larger distance sum)."""
    q = orc.sphere_quadrature(dim)[:, :3]
    for i in range(1, len(q)):
        def key(j):
            d2 = [float(np.float32(np.sum((q[k] - q[j]) ** 2))) for k in range(i)]
            return (min(d2), sum(d2))
        best = max(key(j) for j in range(i, len(q)))
        assert key(i)[0] == best[0]


def _grid(dim, n):
    io = [-v for v in n]  # center_origin for even n
    return dim, n, io


def test_uniform_medium_is_scalar():
    dim, n, io = _grid(3, [8, 8, 8])
    rows = orc.eps_average(dim, n, io, 10.0, 0, [[0, 4.0, 0, 0, 0, 9, 9, 9]], 1.0)
    assert np.all(rows[0] == 0.25) and np.all(rows[1] == 0) and np.all(rows[2] == 0)


def test_maxeval_zero_is_centre_sample():
    dim, n, io = _grid(2, [12, 12, 0])
    objs = [[1, 6.0, 0.013, -0.021, 0, 0.33, 0, 0]]
    for c in (0, 1, 2):
        rows = orc.eps_average(dim, n, io, 10.0, c, objs, 2.0, use_averaging=False)
        o = orc.Oracle(2, n, 10.0, io=io)
        x, y = o.coords(c)
        # the pixel centre is (min + max) * 0.5 of dV(here), the Yee point itself here
        eps = np.where((x - 0.013) ** 2 + (y + 0.021) ** 2 <= 0.33 ** 2, 6.0, 2.0)
        assert np.array_equal(rows[c], 1.0 / eps)
        for d in range(3):
            if d != c:
                assert np.all(rows[d] == 0)


def _plane_means(xmin, dx, x0, e1, e2, tol=1e-4, maxeval=100000):
    """eff_chi1inv_row's refinement loop (ms = 10, 20, 40, ...; 3-D stopping rule)
    for a pixel cut by the plane x = x0 (eps e1 below): the sample grid's mean eps
    and mean 1/eps, which only depend on the x samples."""
    meps = minveps = 1.0
    old_m = old_i = 0.0
    ms, it = 10, 0
    while abs(meps - old_m) > tol * abs(old_m) and abs(minveps - old_i) > tol * abs(old_i):
        old_m, old_i = meps, minveps
        xs = xmin + np.arange(ms) * dx / ms
        f = np.mean(xs <= x0)
        meps, minveps = f * e1 + (1 - f) * e2, f / e1 + (1 - f) / e2
        ms *= 2
        it += ms ** 3
        if it >= maxeval:
            break
    return meps, minveps


def test_planar_interface_kottke_tensor():
    """A half space x < x0 (eps1) in eps2: pixels cut by the plane get the
    harmonic mean along x and the arithmetic mean along y / z (the projection
    tensor with n = x), with the sampled fill fraction of the 10^3 grid."""
    dim, n, io = _grid(3, [10, 10, 10])
    a, e1, e2, x0 = 10.0, 12.0, 2.0, 0.0137
    objs = [[0, e1, x0 - 50.0, 0, 0, 100.0, 100.0, 100.0]]
    o = orc.Oracle(3, n, a, io=io)
    for c in range(3):
        rows = orc.eps_average(dim, n, io, a, c, objs, e2, tol=1e-4, maxeval=100000)
        x, y, z = o.coords(c)
        cut = np.abs(x - x0) < 0.5 / a
        assert cut.sum() > 0
        want = np.empty_like(x)
        for idx in np.flatnonzero(cut.ravel()):
            meps, minveps = _plane_means(float(x.ravel()[idx]) - 0.5 / a, 1.0 / a, x0, e1, e2)
            want.ravel()[idx] = minveps if c == 0 else 1.0 / meps
        diag = rows[c]
        # farther than the normal_vector sphere (radius = one pixel) from the plane: the
        # scalar value exactly; within it but with a uniform pixel: the scalar value up to
        # the rounding of the 1000-sample sums
        far = np.abs(x - x0) >= 1.0 / a
        scal = np.where(x <= x0, 1 / e1, 1 / e2)
        assert np.array_equal(diag[far], scal[far])
        assert np.allclose(diag[~cut], scal[~cut], rtol=1e-13, atol=0)
        assert np.allclose(diag[cut], want[cut], rtol=1e-12, atol=0)
        for d in range(3):
            if d != c:
                assert np.max(np.abs(rows[d])) < 1e-12


def test_sphere_tensor_properties():
    """Averaged tensor over a sphere: rows of the projection form
    n_r n_i (minveps - 1/meps) + delta_ri / meps, bounded by the two media."""
    dim, n, io = _grid(3, [12, 12, 12])
    e1, e2 = 9.0, 1.5
    objs = [[1, e1, 0.017, -0.012, 0.009, 0.41, 0, 0]]
    for c in range(3):
        rows = orc.eps_average(dim, n, io, 10.0, c, objs, e2, maxeval=20000)
        diag = rows[c]
        assert np.all(diag >= 1 / e1 - 1e-12) and np.all(diag <= 1 / e2 + 1e-12)  # sums of 1/eps round
        mixed = (np.abs(diag - 1 / e1) > 1e-9) & (np.abs(diag - 1 / e2) > 1e-9)
        assert mixed.sum() > 50
        off = [rows[d] for d in range(3) if d != c]
        assert max(np.max(np.abs(r)) for r in off) > 1e-3  # the normal is oblique somewhere
        assert max(np.max(np.abs(r)) for r in off) < (1 / e2 - 1 / e1)


def test_oracle_set_epsilon_geometry_drops_trivial_rows():
    o = orc.Oracle(2, [10, 10, 0], 10.0, io=(-10, -10, 0))
    o.set_epsilon_geometry([[0, 3.0, 0.0, 0.0, 0.0, 0.25, 0.6, 0.0]], 1.0)
    # runs a step without complaint (rows accepted per chunk)
    o.add_gaussian_source(2, 0.3, 3.0, 0.0, 20.0, (0.0, 0.0, 0.0), 1.0)
    o.step(5)


def test_simulation_objects_match_geometry_records():
    """Simulation's Block / Sphere / Cylinder (used for non-averaged properties) and
    their mnl_structure_set_epsilon_geometry records (used for averaged epsilon)
    describe the same regions: without averaging the rows are 1/eps at the pixel
    centres, which is what the objects' contains() gives at the Yee points."""
    import meep_nl_amd as mp
    geom = [mp.Block(size=mp.Vector3(1e20, 0.43, 0.37), material=mp.Medium(epsilon=6.0)),
            mp.Sphere(0.52, center=mp.Vector3(0.121, -0.087, 0.053), material=mp.Medium(epsilon=9.0)),
            mp.Cylinder(0.18, height=0.9, axis=mp.Vector3(0, 0, 1),
                        center=mp.Vector3(-0.31, 0.27, 0.013), material=mp.Medium(epsilon=2.5)),
            mp.Cylinder(0.15, height=1.1, axis=mp.Vector3(1, 0, 0),
                        center=mp.Vector3(0.017, 0.33, -0.29), material=mp.Medium(epsilon=3.5))]
    objs = [g.geo_record(g.material.epsilon_diag.x) for g in geom]
    n, io = [22, 20, 24], [-22, -20, -24]
    o = orc.Oracle(3, n, 10.0, io=io)
    for c in range(3):
        rows = orc.eps_average(3, n, io, 10.0, c, objs, 1.7, use_averaging=False)
        x, y, z = o.coords(c)
        eps = np.full(x.shape, 1.7)
        for g in geom:
            eps = np.where(g.contains(x, y, z), g.material.epsilon_diag.x, eps)
        assert np.array_equal(rows[c], 1.0 / eps), c
