"""Seeded random configurations, GPU against the CPU oracle bit for bit on every array:
grid shape and origin, PML thickness on a random subset of faces, dielectric boxes (the
chi1inv palette), a Lorentzian box (polarization chunks), a Kerr box, one to three
Gaussian point sources on E or H components (H sources: the unfused path), random
initial D / B, and the step count are drawn from the seed.  One GPU for every seed, two
in-process slabs where the grid allows.  Complements the hand-built scenarios of
tests/test_gpu_parity.py with the combinations nobody wrote down."""
import numpy as np
import pytest

from scenarios import ALL_COMPS, E_COMPS, GroupSim, ProductSim, make_oracle, random_init, vol

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

SEEDS = list(range(80))


def _box(rng, sizes):
    lo, hi = [], []
    for L in sizes:
        a, b = sorted(rng.uniform(-0.5 * L, 0.5 * L, 2))
        lo.append(a)
        hi.append(b + 0.15)
    return lo, hi


def _inside(o, c, lo, hi):
    xyz = o.coords(c)
    m = np.ones_like(xyz[0], dtype=bool)
    for d, v in enumerate(xyz):
        m &= (v >= lo[d]) & (v <= hi[d])
    return m


def build(make, seed):
    rng = np.random.default_rng(1000 + seed)
    sizes = [float(rng.choice([2.0, 2.7, 3.3, 4.1, 5.2, 6.4])) for _ in range(3)]
    o = vol(make, 3, sizes, 10, center_origin=bool(rng.integers(0, 2)))
    dpml = float(rng.choice([0.0, 0.3, 0.5, 0.8]))
    if dpml > 0:
        dirs = tuple(d for d in range(3) if rng.random() < 0.75 and sizes[d] > 2 * dpml + 0.6)
        sides = (0, 1) if rng.random() < 0.7 else (int(rng.integers(0, 2)),)
        if dirs:
            o.add_pml(dpml, dirs=dirs, sides=sides)
    if rng.random() < 0.6:  # dielectric boxes
        inv = {c: np.ones(o.shape()) for c in E_COMPS}
        for _ in range(int(rng.integers(1, 4))):
            lo, hi = _box(rng, sizes)
            eps = float(rng.uniform(1.5, 12.0))
            for c in E_COMPS:
                inv[c] = np.where(_inside(o, c, lo, hi), 1.0 / eps, inv[c])
        for c in E_COMPS:
            o.set_chi1inv(c, c, inv[c])
    if rng.random() < 0.25:  # Lorentzian box
        lo, hi = _box(rng, sizes)
        s = float(rng.uniform(0.2, 1.0))
        o.add_lorentzian(float(rng.uniform(0.6, 1.4)), float(rng.uniform(0.02, 0.2)),
                         [np.where(_inside(o, c, lo, hi), s, 0.0) for c in E_COMPS])
    if rng.random() < 0.2:  # Kerr box
        lo, hi = _box(rng, sizes)
        for c in E_COMPS:
            o.set_chi3(c, np.where(_inside(o, c, lo, hi), 1e-2, 0.0))
    for _ in range(int(rng.integers(1, 4))):
        comp = int(rng.choice([0, 1, 2, 0, 1, 2, 3, 4, 5]))
        cen = o.center()  # the cell is [0, L] without center_origin
        pos = tuple(float(cen[d] + rng.uniform(-0.4, 0.4) * L) for d, L in enumerate(sizes))
        f = float(rng.uniform(0.15, 0.5))
        end = float(rng.uniform(20.0, 100.0))  # start = -end: the pulse peaks at t = 0
        o.add_gaussian_source(comp, f, float(rng.uniform(2.0, 10.0)), -end, end, pos,
                              float(rng.uniform(0.5, 2.0)))
    if rng.random() < 0.5:
        random_init(o, (6, 7, 8, 9, 10, 11), seed=seed)
    steps = int(rng.integers(3, 31))
    o.step(steps)
    return o, sizes


@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_one_gpu(seed):
    p, _ = build(ProductSim, seed)
    o, _ = build(make_oracle, seed)
    assert p.t == o.t
    assert any(np.any(o.get_array(c) != 0) for c in ALL_COMPS)  # not a trivial comparison
    for c in ALL_COMPS:
        a, b = p.get_array(c), o.get_array(c)
        assert a.shape == b.shape, c
        assert np.array_equal(a, b), (seed, c, float(np.max(np.abs(a - b))))


@pytest.mark.parametrize("seed", SEEDS[::4])
def test_fuzz_two_slabs(seed):
    p, _ = build(GroupSim, seed)
    o, _ = build(make_oracle, seed)
    for c in ALL_COMPS:
        a, b = p.get_array(c), o.get_array(c)
        assert np.array_equal(a, b), (seed, c, float(np.max(np.abs(a - b))))


# ---- richer family: conductivity (D and B), chi(2) (the Newton-Raphson E update), an
# integrated source, and DFT flux planes compared as fluxes and per-point DFT arrays
SEEDS_RICH = list(range(40))
FREQS = [0.2, 0.27, 0.33]


def build_rich(make, seed):
    rng = np.random.default_rng(5000 + seed)
    sizes = [float(rng.choice([2.0, 2.7, 3.3, 4.1])) for _ in range(3)]
    o = vol(make, 3, sizes, 10, center_origin=True)
    if rng.random() < 0.7:
        o.add_pml(0.5, dirs=tuple(d for d in range(3) if sizes[d] > 1.6))
    if rng.random() < 0.5:
        lo, hi = _box(rng, sizes)
        eps = float(rng.uniform(1.5, 6.0))
        for c in E_COMPS:
            o.set_chi1inv(c, c, np.where(_inside(o, c, lo, hi), 1.0 / eps, 1.0))
    if rng.random() < 0.5:  # conductivity on D and / or B
        for c in ((6, 7, 8) if rng.random() < 0.5 else (9, 10, 11)):
            lo, hi = _box(rng, sizes)
            o.set_conductivity(c, np.where(_inside(o, c, lo, hi), float(rng.uniform(0.1, 1.5)), 0.0))
    if rng.random() < 0.35:  # chi(2): Newton-Raphson E update
        lo, hi = _box(rng, sizes)
        for c in E_COMPS:
            o.set_chi2(c, np.where(_inside(o, c, lo, hi), 0.5, 0.0))
    for k in range(int(rng.integers(1, 3))):
        comp = int(rng.choice([0, 1, 2]))
        pos = tuple(float(rng.uniform(-0.3, 0.3) * L) for L in sizes)
        o.add_gaussian_source(comp, 0.3, 4.0, 0.0, 40.0, pos, float(rng.uniform(0.5, 2.0)),
                              is_integrated=bool(k == 1 and rng.random() < 0.5))
    hs = []
    if rng.random() < 0.6:  # an x-normal and a z-normal flux plane
        x = float(rng.uniform(-0.3, 0.3) * sizes[0])
        z = float(rng.uniform(-0.3, 0.3) * sizes[2])
        hy, hz, hx = 0.45 * sizes[1], 0.45 * sizes[2], 0.45 * sizes[0]
        hs.append(o.add_dft_flux([([x, -hy, -hz], [x, hy, hz], 0, 1.0)], FREQS, 1))
        hs.append(o.add_dft_flux([([-hx, -hy, z], [hx, hy, z], 2, 1.0)], FREQS, 1))
    o.step(int(rng.integers(5, 31)))
    return o, hs


@pytest.mark.parametrize("seed", SEEDS_RICH)
def test_fuzz_rich(seed):
    p, hp = build_rich(ProductSim, seed)
    o, ho = build_rich(make_oracle, seed)
    assert any(np.any(o.get_array(c) != 0) for c in ALL_COMPS)
    for c in ALL_COMPS:
        a, b = p.get_array(c), o.get_array(c)
        assert np.array_equal(a, b), (seed, c, float(np.max(np.abs(a - b))))
    for a, b in zip(hp, ho):
        assert np.array_equal(np.asarray(p.flux(a)), np.asarray(o.flux(b))), seed
        for which in (0, 1):
            assert np.array_equal(p.dft_data(a, which), o.dft_data(b, which)), (seed, which)


# ---- 2-D family (TE and TM components together, the unfused 2-D kernels)
@pytest.mark.parametrize("seed", list(range(30)))
def test_fuzz_2d(seed):
    def build2(make):
        rng = np.random.default_rng(9000 + seed)
        sizes = [float(rng.choice([3.0, 4.5, 6.0, 8.3])) for _ in range(2)]
        o = vol(make, 2, sizes, 10, center_origin=bool(rng.integers(0, 2)))
        if rng.random() < 0.7:
            o.add_pml(float(rng.choice([0.5, 1.0])), dirs=(0, 1))
        if rng.random() < 0.6:
            lo, hi = _box(rng, sizes + [1.0])
            eps = float(rng.uniform(1.5, 12.0))
            for c in E_COMPS:
                xy = o.coords(c)
                m = (xy[0] >= lo[0]) & (xy[0] <= hi[0]) & (xy[1] >= lo[1]) & (xy[1] <= hi[1])
                o.set_chi1inv(c, c, np.where(m, 1.0 / eps, 1.0))
        for _ in range(int(rng.integers(1, 4))):
            comp = int(rng.choice([0, 1, 2, 3, 4, 5]))
            cen = o.center()
            pos = tuple(float(cen[d] + rng.uniform(-0.4, 0.4) * L) for d, L in enumerate(sizes))
            o.add_gaussian_source(comp, float(rng.uniform(0.15, 0.5)), 5.0, -60.0, 60.0, pos, 1.0)
        o.step(int(rng.integers(10, 80)))
        return o
    p, o = build2(ProductSim), build2(make_oracle)
    assert any(np.any(o.get_array(c) != 0) for c in ALL_COMPS if o.get_array(c).size)
    for c in ALL_COMPS:
        a, b = p.get_array(c), o.get_array(c)
        assert np.array_equal(a, b), (seed, c, float(np.max(np.abs(a - b))) if a.size else 0)


# ---- physics family: anisotropic Lorentzian sigma (diagonal + one symmetric off-diagonal
# pair), upstream Meep's Pade chi2 / chi3 mode, mu boxes with a magnetic Lorentzian
@pytest.mark.parametrize("seed", list(range(30)))
def test_fuzz_physics(seed):
    def build3(make):
        rng = np.random.default_rng(13000 + seed)
        sizes = [float(rng.choice([2.0, 2.7, 3.3])) for _ in range(3)]
        o = vol(make, 3, sizes, 10, center_origin=True)
        if rng.random() < 0.7:
            o.add_pml(0.5)
        kind = int(rng.integers(0, 3))
        lo, hi = _box(rng, sizes)
        if kind == 0:  # anisotropic sigma
            a, b = sorted(rng.choice(3, 2, replace=False))
            sig = [[None] * 3 for _ in range(3)]
            v = float(rng.uniform(0.05, 0.15))
            for c in E_COMPS:
                m = _inside(o, c, lo, hi)
                sig[c][c] = np.where(m, float(rng.uniform(0.2, 0.6)), 0.0)
                h = 0.05  # off-diagonal entries half a pixel back along c
                xyz = [q - h * (d == c) for d, q in enumerate(o.coords(c))]
                ms = np.ones_like(xyz[0], dtype=bool)
                for d in range(3):
                    ms &= (xyz[d] >= lo[d]) & (xyz[d] <= hi[d])
                if c == a:
                    sig[c][b] = np.where(ms, v, 0.0)
                if c == b:
                    sig[c][a] = np.where(ms, v, 0.0)
            o.add_lorentzian_tensor(float(rng.uniform(0.8, 1.3)), 0.05, sig)
        elif kind == 1:  # upstream nonlinear mode
            o.set_upstream_nl(True)
            for c in E_COMPS:
                m = _inside(o, c, lo, hi)
                o.set_chi1inv(c, c, np.where(m, 1 / 2.25, 1.0))
                o.set_chi3(c, np.where(m, 2e-2, 0.0))
                if rng.random() < 0.5:
                    o.set_chi2(c, np.where(m, 3e-2, 0.0))
        else:  # mu box and a magnetic Lorentzian
            mu = float(rng.uniform(1.5, 4.0))
            o.set_mu_fn(lambda x, y, z: np.where((x >= lo[0]) & (x <= hi[0]) & (y >= lo[1]) &
                                                 (y <= hi[1]) & (z >= lo[2]) & (z <= hi[2]), mu, 1.0))
            if rng.random() < 0.6:
                o.add_magnetic_lorentzian(float(rng.uniform(0.8, 1.3)), 0.1,
                                          [np.where(_inside(o, c, lo, hi), 0.3, 0.0)
                                           for c in (3, 4, 5)])
        for _ in range(int(rng.integers(1, 3))):
            pos = tuple(float(rng.uniform(-0.3, 0.3) * L) for L in sizes)
            o.add_gaussian_source(int(rng.integers(0, 3)), 0.3, 4.0, 0.0, 40.0, pos,
                                  float(rng.uniform(1.0, 20.0)))
        o.step(int(rng.integers(5, 31)))
        return o
    p, o = build3(ProductSim), build3(make_oracle)
    assert any(np.any(o.get_array(c) != 0) for c in ALL_COMPS)
    for c in ALL_COMPS:
        a, b = p.get_array(c), o.get_array(c)
        assert np.array_equal(a, b), (seed, c, float(np.max(np.abs(a - b))))
