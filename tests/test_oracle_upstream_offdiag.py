"""Off-diagonal chi1inv in upstream mode (the OFFDIAG averages the fork comments
out: src/step_generic.cpp:597-598, 617, 632, 659, 772, 823, 844), oracle side.

Parity pin: no reference test exercises these branches (the fork disables them
and tests/aniso_disp.cpp needs Bloch boundaries), so the oracle's restatement
is checked against a second, array-level restatement of the same source lines
(numpy, one step from random fields), plus exact properties: linearity (doubled
sources give bitwise doubled fields) and the fork mode ignoring the rows.
"""
import numpy as np

import scenarios as S
from scenarios import make_oracle

D_OF = {0: 6, 1: 7, 2: 8}  # E component -> D component


def _offdiag_cell(upstream=True, seed=3):
    o = S.vol(make_oracle, 3, [1.6, 1.4, 1.2], 10, center_origin=True)
    if upstream:
        o.set_upstream_nl(True)
    rng = np.random.default_rng(seed)
    shp = o.shape()
    u = {}
    for c in range(3):
        u[c, c] = 0.4 + 0.2 * rng.random(shp)
    for c, d in ((0, 1), (1, 2), (0, 2)):
        v = 0.05 * rng.standard_normal(shp)
        u[c, d] = u[d, c] = v
    for (c, d), v in u.items():
        o.set_chi1inv(c, d, v)
    S.random_init(o, (6, 7, 8, 9, 10, 11), seed=11)
    return o, u


def _offd(uo, g, s_ax, sx_ax):
    """0.25 * ((g[i] + g[i - sx]) * u[i] + (g[i + s] + g[(i + s) - sx]) * u[i + s]) on
    the interior block [1:-1]^3 (s / sx unit strides along axes s_ax / sx_ax)."""
    def sh(a, ds, dx):  # a[i + ds*s - dx*sx] on the interior block
        idx = [slice(1, -1)] * 3
        off = [0, 0, 0]
        off[s_ax] += ds
        off[sx_ax] -= dx
        idx = tuple(slice(1 + o_, a.shape[k] - 1 + o_) for k, o_ in enumerate(off))
        return a[idx]
    return 0.25 * ((sh(g, 0, 0) + sh(g, 0, 1)) * sh(uo, 0, 0) +
                   (sh(g, 1, 0) + sh(g, 1, 1)) * sh(uo, 1, 0))


def test_offdiag_e_update_matches_source_formula():
    """After one step, every interior E point equals
    g*u + OFFDIAG(u1, g1, s1) + OFFDIAG(u2, g2, s2) of the new D (3x3, no chi:
    src/step_generic.cpp:823 with the fork's comment removed), bitwise."""
    o, u = _offdiag_cell()
    o.step(1)
    D = {c: o.get_array(D_OF[c]) for c in range(3)}
    inner = (slice(1, -1),) * 3
    for c in range(3):
        d1, d2 = (c + 1) % 3, (c + 2) % 3
        want = D[c][inner] * u[c, c][inner]
        want = want + _offd(u[c, d1], D[d1], c, d1)
        want = want + _offd(u[c, d2], D[d2], c, d2)
        got = o.get_array(c)[inner]
        np.testing.assert_array_equal(got, want)


def test_offdiag_ignored_in_fork_mode():
    """The fork's step_update_EDHB keeps OFFDIAG commented out (623/644/823/844):
    without chi2 the off-diagonal rows change nothing there."""
    a, _ = _offdiag_cell(upstream=False)
    b = S.vol(make_oracle, 3, [1.6, 1.4, 1.2], 10, center_origin=True)
    rng = np.random.default_rng(3)
    for c in range(3):
        b.set_chi1inv(c, c, 0.4 + 0.2 * rng.random(b.shape()))
    S.random_init(b, (6, 7, 8, 9, 10, 11), seed=11)
    a.step(3)
    b.step(3)
    for c in range(12):
        np.testing.assert_array_equal(a.get_array(c), b.get_array(c))


def test_offdiag_upstream_linear_scaling():
    """No chi2/chi3: the upstream OFFDIAG update is linear, so doubled sources give
    bitwise doubled fields (PML, Lorentzian, integrated source included)."""
    a = S.sc_upstream_nl_3d(make_oracle, steps=30, chi2=False, chi3=False, offdiag=True)
    b = S.sc_upstream_nl_3d(make_oracle, steps=30, chi2=False, chi3=False, offdiag=True, scale=2.0)
    for c in range(12):
        np.testing.assert_array_equal(2.0 * a.get_array(c), b.get_array(c))
    # and the rows act: the same run without them differs
    n = S.sc_upstream_nl_3d(make_oracle, steps=30, chi2=False, chi3=False, offdiag=False)
    assert not np.array_equal(a.get_array(0), n.get_array(0))
