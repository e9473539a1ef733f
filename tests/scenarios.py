"""Identical scenarios for the CPU oracle and the HIP product (parity tests).

Both backends expose the same small interface (add_pml, set_chi1inv,
set_chi2, set_chi3, add_lorentzian, add_gaussian_source,
add_continuous_source, legacy_point_source, step, get_field, get_array,
center, t, dt, time, round_time).  Sizes are chosen so the oracle finishes
in seconds.
"""
import math

import numpy as np

from oracle import oracle as orc

E_COMPS = (0, 1, 2)
ALL_COMPS = tuple(range(12))


def make_oracle(dim, n, a, courant=0.5, io=(0, 0, 0)):
    return orc.Oracle(dim, n, a, courant, io)


class ProductSim:
    """Adapter: meep_nl_amd.core Structure + Fields behind the oracle interface."""

    def __init__(self, dim, n, a, courant=0.5, io=(0, 0, 0)):
        from meep_nl_amd import core
        self.core = core
        self.gv = core.GridVolume(dim, n, a, io)
        self.s = core.Structure(self.gv, courant)
        self.f = None
        self.dim = dim

    def _fields(self):
        if self.f is None:
            self.f = self.core.Fields(self.s)
        return self.f

    def shape(self):
        return self.gv.shape()

    def coords(self, c):
        return self.gv.coords(c)

    def center(self):
        return self.gv.center()

    def add_pml(self, *a, **k):
        self.s.add_pml(*a, **k)

    def set_chi1inv(self, c, d, arr):
        self.s.set_chi1inv(c, d, arr)

    def set_chi2(self, c, arr):
        self.s.set_chi2(c, arr)

    def set_epsilon_geometry(self, objs, default_eps=1.0, use_averaging=True, tol=1e-4,
                             maxeval=100000):
        self.s.set_epsilon_geometry(objs, default_eps, use_averaging, tol, maxeval)

    def set_chi3(self, c, arr):
        self.s.set_chi3(c, arr)

    def set_mu_fn(self, fn):
        self.s.set_mu_fn(fn)

    def add_magnetic_lorentzian(self, *a, **k):
        self.s.add_magnetic_lorentzian(*a, **k)

    def set_conductivity(self, c, arr):
        self.s.set_conductivity(c, arr)

    def add_lorentzian_tensor(self, *a, **k):
        self.s.add_lorentzian_tensor(*a, **k)

    def add_lorentzian(self, *a, **k):
        self.s.add_lorentzian(*a, **k)

    def add_gaussian_source(self, *a, **k):
        self._fields().add_gaussian_source(*a, **k)

    def add_continuous_source(self, *a, **k):
        self._fields().add_continuous_source(*a, **k)

    def add_volume_source(self, *a, **k):
        self._fields().add_volume_source(*a, **k)

    def add_gaussian_volume_source(self, *a, **k):
        self._fields().add_gaussian_volume_source(*a, **k)

    def add_custom_volume_source(self, *a, **k):
        self._fields().add_custom_volume_source(*a, **k)

    def add_custom_source(self, *a, **k):
        self._fields().add_custom_source(*a, **k)

    def legacy_point_source(self, *a, **k):
        self._fields().legacy_point_source(*a, **k)

    def require_component(self, c):
        self._fields().require_component(c)

    def initialize_field(self, c, values):
        self._fields().initialize_field(c, values)

    def field_energy(self):
        return self._fields().field_energy()

    def electric_energy_in_box(self, vmin=None, vmax=None):
        return self._fields().electric_energy_in_box(vmin, vmax)

    def magnetic_energy_in_box(self, vmin=None, vmax=None):
        return self._fields().magnetic_energy_in_box(vmin, vmax)

    def field_energy_in_box(self, vmin=None, vmax=None):
        return self._fields().field_energy_in_box(vmin, vmax)

    def step(self, n=1):
        self._fields().step(n)

    def get_field(self, c, p):
        return self._fields().get_field(c, p)

    def get_array(self, c):
        return self._fields().get_array(c)

    @property
    def t(self):
        return self._fields().t

    @property
    def dt(self):
        return self._fields().dt

    def time(self):
        return self._fields().time()

    def round_time(self):
        return self._fields().round_time()

    def nr_random_fallbacks(self):
        return self._fields().nr_fallbacks()

    def add_dft_flux(self, regions, freqs, decimation=0):
        return self._fields().add_dft_flux(regions, freqs, decimation)

    def set_upstream_nl(self, on=True):
        self.s.set_nonlinear_mode("upstream" if on else "fork")

    def flux(self, h):
        return self._fields().flux(h)

    def dft_data(self, h, which):
        return self._fields().dft_data(h, which)

    def dft_decimation(self, h):
        return self._fields().dft_decimation(h)

    def add_dft_fields(self, comps, vmin, vmax, freqs, yee_grid=False, decimation=0):
        return self._fields().add_dft_fields(comps, vmin, vmax, freqs, yee_grid, decimation)

    def dft_array(self, h, comp, num_freq):
        return self._fields().dft_array(h, comp, num_freq)

    def dump(self, path):
        self._fields().dump(path)

    def get_array_slice(self, c, lo, hi, snap=False):
        return self._fields().get_array_slice(c, lo, hi, snap)

    def load(self, path):
        self._fields().load(path)


class GroupSim(ProductSim):
    """nranks z-slabs (y-slabs in 2-D) of one grid on one GPU, one host thread per
    slab (mnl_fields_create_local): the multi-GPU decomposition and halo exchange
    with the RCCL transport swapped for device copies."""

    NRANKS = 2

    def __init__(self, dim, n, a, courant=0.5, io=(0, 0, 0)):
        super().__init__(dim, n, a, courant, io)
        self.nranks = self.NRANKS
        self.fs = None

    def _all(self):
        if self.fs is None:
            self.hub = self.core.LocalHub(self.nranks)
            self.fs = [self.core.Fields(self.s, rank=r, nranks=self.nranks, hub=self.hub)
                       for r in range(self.nranks)]
        return self.fs

    def _fields(self):
        return self._all()[0]

    def _par(self, fn):
        import threading
        out = [None] * self.nranks
        err = []

        def run(r):
            try:
                out[r] = fn(self.fs[r])
            except Exception as e:  # noqa: BLE001
                err.append(e)
        th = [threading.Thread(target=run, args=(r,)) for r in range(self.nranks)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if err:
            raise err[0]
        return out

    def add_gaussian_source(self, *a, **k):
        for f in self._all():
            f.add_gaussian_source(*a, **k)

    def add_continuous_source(self, *a, **k):
        for f in self._all():
            f.add_continuous_source(*a, **k)

    def add_volume_source(self, *a, **k):
        for f in self._all():
            f.add_volume_source(*a, **k)

    def add_gaussian_volume_source(self, *a, **k):
        for f in self._all():
            f.add_gaussian_volume_source(*a, **k)

    def add_custom_volume_source(self, *a, **k):
        for f in self._all():
            f.add_custom_volume_source(*a, **k)

    def legacy_point_source(self, *a, **k):
        for f in self._all():
            f.legacy_point_source(*a, **k)

    def get_array_slice(self, c, lo, hi, snap=False):  # collective: every rank gets the slice
        out = self._par(lambda f: f.get_array_slice(c, lo, hi, snap))
        for o in out[1:]:
            assert np.array_equal(o, out[0])
        return out[0]

    def add_custom_source(self, *a, **k):  # every rank adds every source (SPMD)
        for f in self._all():
            f.add_custom_source(*a, **k)

    def require_component(self, c):
        for f in self._all():
            f.require_component(c)

    def initialize_field(self, c, values):  # collective (ghost exchange)
        self._all()
        self._par(lambda f: f.initialize_field(c, values))

    def _energy_all(self, name, *a):  # collective: every rank returns the summed energy
        self._all()
        vals = self._par(lambda f: getattr(f, name)(*a))
        assert all(v == vals[0] for v in vals)
        return vals[0]

    def field_energy(self):
        return self._energy_all("field_energy")

    def electric_energy_in_box(self, vmin=None, vmax=None):
        return self._energy_all("electric_energy_in_box", vmin, vmax)

    def magnetic_energy_in_box(self, vmin=None, vmax=None):
        return self._energy_all("magnetic_energy_in_box", vmin, vmax)

    def field_energy_in_box(self, vmin=None, vmax=None):
        return self._energy_all("field_energy_in_box", vmin, vmax)

    def step(self, n=1):
        self._all()
        self._par(lambda f: f.step(n))

    def get_field(self, c, p):
        self._all()
        vals = self._par(lambda f: f.get_field(c, p))
        assert all(v == vals[0] for v in vals)
        return vals[0]

    def get_array(self, c):
        return sum(f.get_array(c) for f in self._all())

    def nr_random_fallbacks(self):
        return sum(f.nr_fallbacks() for f in self._all())

    def add_dft_flux(self, regions, freqs, decimation=0):
        hs = [f.add_dft_flux(regions, freqs, decimation) for f in self._all()]
        assert all(h == hs[0] for h in hs)
        return hs[0]

    def flux(self, h):
        vals = self._par(lambda f: f.flux(h))  # every rank returns the allreduced sum
        assert all(np.array_equal(v, vals[0]) for v in vals)
        return vals[0]

    def dft_data(self, h, which):
        # each point is accumulated by the rank that owns it, the others hold 0
        return sum(f.dft_data(h, which) for f in self._all())

    def add_dft_fields(self, comps, vmin, vmax, freqs, yee_grid=False, decimation=0):
        hs = [f.add_dft_fields(comps, vmin, vmax, freqs, yee_grid, decimation) for f in self._all()]
        assert all(h == hs[0] for h in hs)
        return hs[0]

    def dft_array(self, h, comp, num_freq):
        vals = self._par(lambda f: f.dft_array(h, comp, num_freq))  # collective, summed
        assert all(np.array_equal(v, vals[0]) for v in vals)
        return vals[0]


    def dump(self, path):
        self._all()
        self._par(lambda f: f.dump(path))

    def load(self, path):
        self._all()
        self._par(lambda f: f.load(path))


class GroupSim3(GroupSim):
    NRANKS = 3


def vol(make, dim, sizes, a, center_origin=False, courant=0.5):
    n = [0, 0, 0]
    if dim == 1:
        n[2] = int(sizes[0] * a + 0.5)
    elif dim == 2:
        n[0] = int(sizes[0] * a + 0.5)
        n[1] = int(sizes[1] * a + 0.5)
    else:
        n = [int(s * a + 0.5) for s in sizes]
    io = [-(v - (v & 1)) for v in n] if center_origin else [0, 0, 0]
    return make(dim, n, a, courant, io)


# ------------------------------------------------------------------ scenarios
# Each returns the simulation object after stepping.

def sc_cfg1(make, steps=500):
    """Config 1 (BASELINE configs[0]): 2-D 200x200 vacuum, Ez Gaussian current at the
    origin, metallic walls, real fields."""
    o = vol(make, 2, [20, 20], 10, center_origin=True)
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0, 0), 1.0, is_integrated=False)
    o.step(steps)
    return o


def sc_vacuum_pml_3d(make, L=3.2, steps=60, dpml=1.0):
    """Config 2 shape scaled down: vacuum box + PML on all faces, Ez Gaussian current at
    (0.05,0.05,0.05)."""
    o = vol(make, 3, [L, L, L], 10, center_origin=True)
    o.add_pml(dpml)
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    o.step(steps)
    return o


def sc_c5_small(make, nranks=8, nxy=64, nz_per=16, steps=30):
    """BASELINE configs[4] (C5) decomposition at reduced x-y: vacuum + PML(1.0) on a
    nxy x nxy x (nz_per * nranks) grid at resolution 10 (C5 is 512 x 512 x (128 * 8)),
    z-slab split over nranks ranks (the 10-plane z-PML lies on the end ranks only, the
    interior ranks have two neighbours), Ez Gaussian current at the centre."""
    o = vol(make, 3, [nxy / 10.0, nxy / 10.0, nz_per * nranks / 10.0], 10, center_origin=True)
    o.add_pml(1.0)
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    o.step(steps)
    return o


def sc_c5_full(make, steps=7, log=None):
    """BASELINE configs[4] (C5) at full size: the 512 x 512 x 1024 vacuum + PML(1.0) grid (the
    8-GPU decomposition is 8 z-slabs of 512 x 512 x 128), seeded random D and B everywhere
    (every slab face and PML chunk carries data from the first step on), the Ez Gaussian
    current at the centre (on the middle slab seam), stepped 1 + 6 (the first step unfused
    after initialize_field, then three pairs of steps)."""
    o = vol(make, 3, [51.2, 51.2, 102.4], 10, center_origin=True)
    o.add_pml(1.0)
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    for c in (6, 7, 8, 9, 10, 11):
        rng = np.random.default_rng(7 + 31 * c)
        v = rng.standard_normal(o.shape())
        o.initialize_field(c, v)
        del v
        if log:
            log(f"initialized component {c}")
    o.step(1)
    o.step(steps - 1)
    return o


def plane_checksums(arr):
    """Per plane of the last (z, the slab) axis: the sum over the plane of each value's IEEE
    bit pattern times an odd weight of its (x, y, z) position, mod 2^64.  Entries a rank does
    not own are 0 in its get_array, and every entry has one owner, so the ranks' checksums
    add up (mod 2^64) to the one-rank run's exactly when every entry is bitwise equal (a
    differing, swapped or misplaced value changes its plane's sum)."""
    a = np.ascontiguousarray(arr).view(np.uint64)
    nx, ny, nz = a.shape
    out = np.zeros(nz, dtype=np.uint64)
    ky = (np.arange(ny, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))[:, None]
    kz = (np.arange(nz, dtype=np.uint64) * np.uint64(0xD6E8FEB86659FD93))[None, :]
    with np.errstate(over="ignore"):
        for i in range(nx):
            w = (np.uint64(i) * np.uint64(0xBF58476D1CE4E5B9) + ky + kz) | np.uint64(1)
            out += (a[i] * w).sum(axis=0, dtype=np.uint64)
    return out


def sc_waveguide_3d(make, L=3.2, steps=40, eps=12.0):
    """Config 3 shape scaled down: eps=12 core |y|,|z| < 0.5 along x, PML, no averaging."""
    o = vol(make, 3, [L, L, L], 10, center_origin=True)
    o.add_pml(1.0)
    for c in E_COMPS:
        x, y, z = o.coords(c)
        e = np.where((np.abs(y) < 0.5) & (np.abs(z) < 0.5), eps, 1.0)
        o.set_chi1inv(c, c, 1.0 / e)
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    o.step(steps)
    return o


def sc_big_box_3d(make, sizes=(14.0, 4.1, 15.3), steps=30, dpml=0.7, eps=6.0, extra=None,
                  random_eps=False):
    """Non-cubic grid spanning many fused tiles in x, y and z; dielectric slab across
    the PML boundary; optional callback(o) after half the steps (mode toggles).
    random_eps: seeded random eps in [1, 12] in the slab (thousands of distinct
    chi1inv values: more than the fused kernel's 256-entry palette)."""
    o = vol(make, 3, list(sizes), 10, center_origin=True)
    o.add_pml(dpml)
    for c in E_COMPS:
        x, y, z = o.coords(c)
        inside = (np.abs(y) < 0.8) & (z > -0.4) & (z < 3.0)
        if random_eps:
            rng = np.random.default_rng(1234 + c)
            val = 1.0 / rng.uniform(1.0, 12.0, size=x.shape)
        else:
            val = 1.0 / eps
        o.set_chi1inv(c, c, np.where(inside, val, 1.0))
    o.add_gaussian_source(2, 0.25, 4.0, 0.0, 40.0, (0.37, -0.21, 0.05), 1.0)
    o.add_gaussian_source(0, 0.3, 4.0, 0.0, 40.0, (-3.3, 0.6, 2.15), 0.6)
    o.step(steps // 2)
    if extra:
        extra(o)
    o.step(steps - steps // 2)
    return o


def sc_kerr_lorentz_3d(make, L=3.2, steps=60):
    """Config 4 shape scaled down: slab |z|<0.6 eps 2.25, chi3 1e-2 (inert in the fork),
    Lorentzian(1.1, 0.05, sigma 0.5), PML, Ex Gaussian at z=-1.0, amp 50."""
    o = vol(make, 3, [L, L, L], 10, center_origin=True)
    o.add_pml(1.0)
    sig = []
    for c in E_COMPS:
        x, y, z = o.coords(c)
        inside = np.abs(z) < 0.6
        o.set_chi1inv(c, c, np.where(inside, 1 / 2.25, 1.0))
        o.set_chi3(c, np.where(inside, 1e-2, 0.0))
        sig.append(np.where(inside, 0.5, 0.0))
    o.add_lorentzian(1.1, 0.05, sig)
    o.add_gaussian_source(0, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, -1.0), 50.0)
    o.step(steps)
    return o


def sc_nr_probe(make, c2=0.5, steps=40):
    """SURVEY.md 8(c) chi(2) Newton-Raphson probe (integrated legacy source)."""
    o = vol(make, 3, [1, 1, 1], 10)
    for c in E_COMPS:
        for d in range(3):
            o.set_chi1inv(c, d, np.full(o.shape(), 0.25 if d == c else 1e-3))
        if c2:
            o.set_chi2(c, np.full(o.shape(), c2))
    cen = o.center()
    o.legacy_point_source(2, 0.5, 0.5, 0.0, 3.0, [cen[0] + 0.05, cen[1] + 0.05, cen[2] + 0.05],
                          5.0)
    o.step(steps)
    return o


def sc_nr_wall_lorentz(make, steps=40):
    """chi2 Newton-Raphson and a Lorentzian up to the metallic walls (no PML): the
    reference's chunk updates E on its high wall planes before zeroing them, and
    update_P keeps what it read there; neighbours see that P through D - P."""
    o = vol(make, 3, [1.2, 1.0, 1.4], 10)
    sig = []
    for c in E_COMPS:
        for d in range(3):
            o.set_chi1inv(c, d, np.full(o.shape(), 0.3 if d == c else 2e-3))
        o.set_chi2(c, np.full(o.shape(), 0.1))
        sig.append(np.full(o.shape(), 0.3))
    o.add_lorentzian(1.1, 0.1, sig)
    o.legacy_point_source(2, 0.6, 0.5, 0.0, 3.0, [1.12, 0.93, 1.31], 1.0)
    o.add_gaussian_source(0, 0.5, 4.0, 0.0, 30.0, (0.6, 0.95, 0.7), 0.5)
    o.step(steps)
    return o


def sc_nr_pml_dispersive(make, steps=30):
    """chi2 NR next to a PML with a Lorentzian background and an integrated source
    (exercises the zone tables and the split E / P kernels)."""
    o = vol(make, 3, [2.6, 2.6, 2.6], 10, center_origin=True)
    o.add_pml(0.6)
    sig = []
    for c in E_COMPS:
        x, y, z = o.coords(c)
        inside = (np.abs(x) < 0.5) & (np.abs(y) < 0.5) & (np.abs(z) < 0.5)
        for d in range(3):
            if d == c:
                o.set_chi1inv(c, d, np.where(inside, 0.25, 1.0))
            else:
                o.set_chi1inv(c, d, np.where(inside, 1e-3, 0.0))
        o.set_chi2(c, np.where(inside, 0.5, 0.0))
        sig.append(np.where(np.abs(z) < 0.3, 0.2, 0.0))
    o.add_lorentzian(0.9, 0.1, sig)
    o.legacy_point_source(2, 0.5, 0.5, 0.0, 3.0, (0.05, 0.05, 0.05), 5.0)
    o.step(steps)
    return o


def sc_nr_isrc_seam(make, steps=30):
    """chi2 Newton-Raphson voxels on both sides of a reference chunk seam (the low-z
    PML boundary, z = -0.6) with integrated sources ON the seam: Ex exactly at the
    seam point (owned by the PML chunk) and Ez between the seam's two neighbours.
    The reference subtracts an integrated dipole only in its owner chunk's
    f_minus_p (src/update_eh.cpp:136-146); the NR 4-point averages of the other
    chunk read the ghost D - P without it (src/step_generic.cpp:740-743)."""
    o = vol(make, 3, [2.6, 2.6, 2.6], 10, center_origin=True)
    o.add_pml(0.6)
    for c in E_COMPS:
        x, y, z = o.coords(c)
        inside = (np.abs(x) < 0.5) & (np.abs(y) < 0.5) & (z > -0.95) & (z < 0.3)
        for d in range(3):
            if d == c:
                o.set_chi1inv(c, d, np.where(inside, 0.25, 1.0))
            else:
                o.set_chi1inv(c, d, np.where(inside, 1e-3, 0.0))
        o.set_chi2(c, np.where(inside, 0.5, 0.0))
    o.legacy_point_source(0, 0.5, 0.5, 0.0, 3.0, (0.05, 0.05, -0.6), 5.0)
    o.legacy_point_source(2, 0.45, 0.5, 0.0, 3.0, (0.0, 0.0, -0.57), 4.0)
    o.legacy_point_source(1, 0.4, 0.5, 0.0, 3.0, (-0.03, 0.02, -0.61), 3.0)
    o.step(steps)
    return o


def random_init(o, comps, seed=7, scale=1.0):
    """Seeded random initial fields through initialize_field (src/initialize.cpp:
    135-161) -- every tile, z chunk, PML region and wall of the grid carries data
    from the first step on."""
    for c in comps:
        rng = np.random.default_rng(seed + 31 * c)
        o.initialize_field(c, scale * rng.standard_normal(o.shape()))


def sc_random_fields(make, sizes=(3.2, 3.2, 3.2), steps=12, dpml=1.0, eps=None, comps=(6, 7, 8, 9, 10, 11),
                     kerr_lorentz=False, source=True):
    """Random D and B everywhere (then E, H from them as the reference's
    initialize_field does), optional dielectric core or Kerr + Lorentzian slab,
    PML, a Gaussian source; stepped."""
    o = vol(make, 3, list(sizes), 10, center_origin=True)
    if dpml:
        o.add_pml(dpml)
    if kerr_lorentz:  # BASELINE configs[3]: |z| < 2 eps 2.25, chi3 1e-2, Lorentzian(1.1, 0.05, 0.5)
        sig = []
        for c in E_COMPS:
            x, y, z = o.coords(c)
            inside = np.abs(z) < 2.0
            o.set_chi1inv(c, c, np.where(inside, 1 / 2.25, 1.0))
            o.set_chi3(c, np.where(inside, 1e-2, 0.0))
            sig.append(np.where(inside, 0.5, 0.0))
        o.add_lorentzian(1.1, 0.05, sig)
    elif eps:
        for c in E_COMPS:
            x, y, z = o.coords(c)
            o.set_chi1inv(c, c, np.where((np.abs(y) < 0.5) & (np.abs(z) < 0.5), 1.0 / eps, 1.0))
    if source:
        if kerr_lorentz:
            o.add_gaussian_source(0, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, -3.0), 50.0)
        else:
            o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    random_init(o, comps)
    o.step(steps)
    return o


def legacy_last_time(freq, width, peaktime, cutoff, a, dt, t=0, magnetic=False):
    """last_source_time() of fields::add_point_source(c, freq, width, peaktime,
    cutoff, ...) (src/sources.cpp:189-211 -> gaussian_src_time, src/meep.hpp:1024)."""
    width = width / freq
    cutoff = (1.0 / a) + cutoff * width
    if peaktime <= 0.0:
        peaktime = t * dt + cutoff
    peaktime += (-dt * 0.5) if magnetic else dt
    st, et = peaktime - cutoff, peaktime + cutoff
    peak, cut = 0.5 * (st + et), (et - st) * 0.5
    while math.exp(-cut * cut / (2 * width * width)) < 1e-100:
        cut *= 0.9
    return float(np.float32(peak + float(np.float32(cut))))


def three_d_test_pml(make, energy_every=None):
    """tests/three_d.cpp:163-194 (test_pml): vol3d(1.5, 1.0, 1.2) @ 10, pml(0.401),
    vacuum, Ez point source (0.8, 0.6, 0, 4) at (0.751, 0.5, 0.601); after the
    source, the field energy must fall below 4e-3 of its value within every 10
    time units up to 31.  Returns (sim, last_energy, [(time, energy)])."""
    o = make(3, [15, 10, 12], 10.0, 0.5, [0, 0, 0])
    o.add_pml(0.401)
    o.legacy_point_source(2, 0.8, 0.6, 0.0, 4.0, (0.751, 0.5, 0.601), 1.0)
    ts = legacy_last_time(0.8, 0.6, 0.0, 4.0, 10.0, 0.05)
    while o.time() < ts:
        o.step()
    last = o.field_energy()
    out, check = [], 10.0
    while o.time() < 3.1 * 10.0:
        o.step()
        if o.time() >= check:
            out.append((o.time(), o.field_energy()))
            check += 10.0
    return o, last, out


def three_d_test_pml_splitting(make):
    """tests/three_d.cpp:196-224 (test_pml_splitting) on one side: vol3d(1.5, 1.0,
    1.2) @ 10, pml(0.3), Ez point source (0.8, 1.6, 0, 4) at (1.099, 0.499, 0.501),
    stepped to t = 31 with field_energy() whenever time() passes 10, 20, 30.
    Returns (sim, [(step, energy)], [probe values])."""
    o = make(3, [15, 10, 12], 10.0, 0.5, [0, 0, 0])
    o.add_pml(0.3)
    o.legacy_point_source(2, 0.8, 1.6, 0.0, 4.0, (1.099, 0.499, 0.501), 1.0)
    nxt, en, probes = 10.0, [], []
    pts = [(0.5, 0.01, 1.0), (0.46, 0.33, 0.33), (1.0, 1.0, 0.33), (1.3, 0.3, 0.15)]
    while o.time() < 31.0:
        o.step()
        if o.t % 25 == 0:
            probes.append([o.get_field(2, p) for p in pts])
        if o.time() > nxt:
            en.append((o.t, o.field_energy()))
            nxt += 10.0
    return o, en, probes


def polariton_energy_1d(make):
    """tests/known_results.cpp:145-155 (polariton_energy): the 1-D polariton of
    sc_polariton_1d and its field_energy() at round_time 10 (golden 0.0863443)."""
    o = sc_polariton_1d(make)
    return o, o.field_energy()


def sc_known_metallic_3d(make):
    o = vol(make, 3, [1, 1, 1], 10)
    o.legacy_point_source(2, 0.2, 3.0, 0.0, 2.0, o.center(), complex(0, -2 * math.pi * 0.2))
    while o.round_time() < 10.0:
        o.step()
    return o


def sc_known_pml_2d(make):
    o = vol(make, 2, [3, 3], 10)
    o.add_pml(1.0)
    o.legacy_point_source(2, 0.2, 3.0, 0.0, 2.0, o.center(), complex(0, -2 * math.pi * 0.2))
    n = 0
    while float(np.float32((n) * (0.5 / 10))) < 30.0:
        n += 1
    o.step(n)
    return o


def sc_polariton_1d(make):
    o = vol(make, 1, [1], 10)
    o.add_lorentzian(0.3, 0.1, [np.full(o.shape(), 7.63), None, None])
    o.legacy_point_source(0, 0.2, 3.0, 0.0, 2.0, o.center(), complex(0, -2 * math.pi * 0.2))
    n = 0
    while float(np.float32(n * (0.5 / 10))) < 10.0:
        n += 1
    o.step(n)
    return o


def sc_te_magnetic_2d(make, steps=80):
    """2-D TE (Hz source, non-integrated magnetic current) + one-sided PML, odd grid."""
    o = vol(make, 2, [2.3, 1.9], 10)
    o.add_pml(0.5, dirs=(0,), sides=(1,))
    o.add_pml(0.4, dirs=(1,), sides=(0,))
    o.add_gaussian_source(5, 0.4, 3.0, 0.0, 30.0, (1.03, 0.77), 2.0)
    o.add_continuous_source(5, 0.3, 2.0, 0.0, 1e20, 3.0, (0.5, 1.2), 0.7)
    o.step(steps)
    return o


def sc_multi_source_3d(make, steps=50):
    """Several sources: off-grid position (interpolation weights), duplicate
    (merged amplitudes), integrated + current, magnetic, near the PML edge."""
    o = vol(make, 3, [3.0, 2.6, 2.2], 10, center_origin=True)
    o.add_pml(0.8)
    o.add_gaussian_source(2, 0.2, 4.0, 0.0, 40.0, (0.013, -0.037, 0.021), 1.0)
    o.add_gaussian_source(2, 0.2, 4.0, 0.0, 40.0, (0.013, -0.037, 0.021), 0.5)
    o.add_gaussian_source(0, 0.25, 4.0, 0.0, 40.0, (0.3, 0.2, -0.1), 1.0, is_integrated=True)
    o.add_gaussian_source(4, 0.3, 4.0, 0.0, 40.0, (-0.2, 0.1, 0.15), complex(0.3, 0.7))
    o.add_gaussian_source(1, 0.3, 4.0, 0.0, 40.0, (1.0, -0.7, 0.6), 1.0)
    o.step(steps)
    return o


def compare_all(a, b, comps=ALL_COMPS):
    """Max abs difference per component between two backends."""
    out = {}
    for c in comps:
        x, y = a.get_array(c), b.get_array(c)
        out[c] = float(np.max(np.abs(x - y))) if x.size else 0.0
    return out


def sc_big_lorentz_3d(make, steps=24, extra=None):
    """Big non-cubic box with a dispersive slab (Lorentzian + eps, across the x/y PML)
    between lean regions: the fused step's polarization box (E stored, P updated in
    the general kernels) next to lean tiles; optional callback(o) mid-run."""
    o = vol(make, 3, [14.0, 4.1, 15.3], 10, center_origin=True)
    o.add_pml(0.7)
    sig = []
    for c in E_COMPS:
        x, y, z = o.coords(c)
        inside = (z > 1.0) & (z < 3.0)
        o.set_chi1inv(c, c, np.where(inside, 1 / 2.25, 1.0))
        sig.append(np.where(inside, 0.5, 0.0))
    o.add_lorentzian(1.1, 0.05, sig)
    o.add_gaussian_source(0, 0.3, 4.0, 0.0, 40.0, (0.05, 0.05, -1.0), 50.0)
    o.add_gaussian_source(2, 0.25, 4.0, 0.0, 40.0, (2.3, -0.4, 4.5), 5.0)
    o.step(steps // 2)
    if extra:
        extra(o)
    o.step(steps - steps // 2)
    return o


# ------------------------------------------------------------------ DFT flux
def flux_box_faces(lo, hi, dim):
    """fields::add_dft_flux_box (src/dft.cpp:831-848): for each direction with extent,
    the max face (+1) then the min face (-1) are prepended to the volume list; the
    regions are returned in the list's iteration order."""
    faces = []
    for d in range(3):
        if dim == 2 and d == 2:
            continue
        if hi[d] - lo[d] > 0:
            mx_lo = list(lo)
            mx_lo[d] = hi[d]
            faces.insert(0, (mx_lo, list(hi), d, 1.0))
            mn_hi = list(hi)
            mn_hi[d] = lo[d]
            faces.insert(0, (list(lo), mn_hi, d, -1.0))
    return faces


FLUX2D_FREQS = [0.230, 0.232, 0.238, 0.241, 0.248, 0.254, 0.256, 0.265, 0.269, 0.270]


def sc_flux_2d(make, xmax=10.0, ymax=10.0, ttot=130.0):
    """tests/flux.cpp:157-225 (flux_2d, second check): voltwo(10,10,8), pml(0.5),
    vacuum (bump2 is 1 at z=0), Ez point source add_point_source(Ez, 0.25, 3.5, 0, 8,
    (xmax/6+0.1, ymax/6+0.3), 1), two concentric DFT flux boxes around it, stepped
    until time() >= 2*ttot.  Returns (sim, handle box1, handle box2)."""
    o = vol(make, 2, [xmax, ymax], 8)
    o.add_pml(0.5)
    o.legacy_point_source(2, 0.25, 3.5, 0.0, 8.0, (xmax / 6 + 0.1, ymax / 6 + 0.3, 0.0), 1.0)
    b1 = flux_box_faces([xmax / 6 - 0.4, ymax / 6 - 0.2, 0], [xmax / 6 + 0.6, ymax / 6 + 0.8, 0], 2)
    b2 = flux_box_faces([xmax / 6 - 0.9, ymax / 6 - 0.7, 0], [xmax / 6 + 1.1, ymax / 6 + 1.3, 0], 2)
    h1 = o.add_dft_flux(b1, FLUX2D_FREQS)
    h2 = o.add_dft_flux(b2, FLUX2D_FREQS)
    n = 0
    while (n + 1) * o.dt < 2 * ttot:  # f.step(); while (f.time() < ttot) ...; ... < 2*ttot
        n += 1
    o.step(n + 1)
    return o, h1, h2


FLUX3D_FREQS = [0.1, 0.15, 0.2, 0.27]


def sc_flux_3d(make, steps=80, sizes=None, lorentz=False, decimation=1, extra=None, freqs=None,
               calls=None):
    """Waveguide (eps 12 core along x) + PML with four DFT flux objects: a box around
    the source (six faces, weights +-1), an x-normal plane across the whole cell
    (through the PML), a z-normal plane inside the lower PML, and a y-direction
    volume region (interpolation weights in all three directions).  Optional
    Lorentzian slab (E stored inside the polarization box in fused mode) and a
    callback(o) at half time.  The last object uses the automatic decimation
    (src/dft.cpp:195-216).  calls: the step counts of the step calls instead (None entries:
    call extra(o) there).  Returns (sim, [handles])."""
    sizes = sizes or [3.2, 3.2, 3.2]
    o = vol(make, 3, sizes, 10, center_origin=True)
    o.add_pml(1.0 if sizes[0] < 4 else 0.7)
    sig = []
    for c in E_COMPS:
        x, y, z = o.coords(c)
        o.set_chi1inv(c, c, np.where((np.abs(y) < 0.5) & (np.abs(z) < 0.5), 1 / 12.0, 1.0))
        sig.append(np.where(np.abs(z - 0.3) < 0.25, 0.5, 0.0))
    if lorentz:
        o.add_lorentzian(1.1, 0.05, sig)
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    o.add_gaussian_source(1, 0.2, 6.0, 0.0, 60.0, (-0.33, 0.12, 0.41), 0.7)
    hx, hy, hz = [0.5 * s for s in sizes]
    FLUX3D_FREQS = list(freqs) if freqs is not None else globals()["FLUX3D_FREQS"]
    hs = [o.add_dft_flux(flux_box_faces([-0.42, -0.37, -0.33], [0.44, 0.51, 0.38], 3),
                         FLUX3D_FREQS, decimation),
          o.add_dft_flux([([0.83, -hy, -hz], [0.83, hy, hz], 0, 1.0)], FLUX3D_FREQS, decimation),
          o.add_dft_flux([([-hx + 0.1, -hy + 0.3, -hz + 0.35], [hx - 0.2, hy - 0.1, -hz + 0.35],
                           2, -0.5)], FLUX3D_FREQS, decimation),
          o.add_dft_flux([([-0.61, -0.23, -0.17], [0.57, 0.29, 0.66], 1, 1.0)], FLUX3D_FREQS,
                         0)]  # automatic decimation
    if calls is not None:
        for n in calls:
            if n is None:
                extra(o)
            else:
                o.step(n)
        return o, hs
    o.step(steps // 2)
    if extra:
        extra(o)
    o.step(steps - steps // 2)
    return o, hs


DFTF_FREQS = [0.12, 0.2]


def sc_dft_fields_3d(make, steps=60, lorentz=False, sizes=None):
    """sc_flux_3d's waveguide + PML with DFT-field objects (fields::add_dft_fields,
    src/dft.cpp:889-903): every E / H component over the whole cell on the centered
    grid; Ez, Hx, Hy on their Yee grids over a box crossing PML chunks; an x-normal
    plane (collapsed to 2-D); a y-z line on the Yee grid (two empty dimensions); a
    flux plane (get_dft_array of a dft_flux).  Returns (sim, [(handle, comps)])."""
    sizes = sizes or [3.2, 3.2, 3.2]
    o = vol(make, 3, sizes, 10, center_origin=True)
    o.add_pml(1.0)
    sig = []
    for c in E_COMPS:
        x, y, z = o.coords(c)
        o.set_chi1inv(c, c, np.where((np.abs(y) < 0.5) & (np.abs(z) < 0.5), 1 / 12.0, 1.0))
        sig.append(np.where(np.abs(z - 0.3) < 0.25, 0.5, 0.0))
    if lorentz:
        o.add_lorentzian(1.1, 0.05, sig)
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    o.add_gaussian_source(1, 0.2, 6.0, 0.0, 60.0, (-0.33, 0.12, 0.41), 0.7)
    hx, hy, hz = [0.5 * s for s in sizes]
    objs = [
        (o.add_dft_fields([0, 1, 2, 3, 4, 5], [-hx, -hy, -hz], [hx, hy, hz], DFTF_FREQS, False, 1),
         [0, 1, 2, 3, 4, 5]),
        (o.add_dft_fields([2, 3, 4], [-1.23, -0.71, -1.3], [0.94, 1.42, 0.57], DFTF_FREQS, True, 1),
         [2, 3, 4]),
        (o.add_dft_fields([1, 5], [0.33, -hy, -hz], [0.33, hy, hz], DFTF_FREQS, False, 0), [1, 5]),
        (o.add_dft_fields([0], [-0.9, 0.27, -0.15], [1.1, 0.27, -0.15], DFTF_FREQS, True, 1), [0]),
        (o.add_dft_flux([([-0.52, -hy, -hz], [-0.52, hy, hz], 0, 1.0)], DFTF_FREQS, 1), [1, 2, 4, 5]),
    ]
    o.step(steps)
    return o, objs


def sc_dft_fields_2d(make, steps=200):
    """2-D TM + TE (Ez and Hz sources) with PML: centered and Yee-grid DFT fields."""
    o = vol(make, 2, [4.0, 3.0], 10)
    o.add_pml(0.7)
    o.add_gaussian_source(2, 0.3, 5.0, 0.0, 50.0, (1.3, 1.1, 0), 1.0)
    o.add_gaussian_source(5, 0.25, 4.0, 0.0, 40.0, (2.6, 1.7, 0), 0.5)
    objs = [
        (o.add_dft_fields([0, 1, 2, 3, 4, 5], [0, 0, 0], [4.0, 3.0, 0], DFTF_FREQS, False, 1),
         [0, 1, 2, 3, 4, 5]),
        (o.add_dft_fields([2, 5, 0], [0.25, 0.4, 0], [3.3, 2.9, 0], DFTF_FREQS, True, 1), [2, 5, 0]),
        (o.add_dft_fields([2, 3], [0.5, 1.55, 0], [3.5, 1.55, 0], DFTF_FREQS, False, 1), [2, 3]),
    ]
    o.step(steps)
    return o, objs


def sc_flux_1d(make, steps=1500, chi3=1e-2):
    """1-D: 20 @ res 20, PML 1, chi3 (inert in the fork), Ex Gaussian near the left;
    transmitted flux plane + a flux 'box' (two points) around the source."""
    o = vol(make, 1, [20.0], 20, center_origin=True)
    o.add_pml(1.0)
    if chi3:
        o.set_chi3(0, np.full(o.shape(), chi3))
    o.add_gaussian_source(0, 1 / 3, 60.0 / 8, 0.0, 75.0, (0, 0, -8.0), 10.0)
    fr = [0.25, 1 / 3, 0.4, 1.0]
    hs = [o.add_dft_flux([([0, 0, 7.5], [0, 0, 7.5], 2, 1.0)], fr, 1),
          o.add_dft_flux(flux_box_faces([0, 0, -8.5], [0, 0, -7.3], 3), fr, 0)]
    o.step(steps)
    return o, hs


def third_harmonic_1d(make, upstream=True, decay=1e-6):
    """python/tests/test_3rd_harm_1d.py on the scenario interface: returns (sim,
    flux(fcen), flux(3 fcen)) after run(until_after_sources=
    stop_when_fields_decayed(50, Ex, pt, decay)) replayed step by step."""
    sz, fcen, dpml, k = 100, 1 / 3.0, 1.0, 1e-2
    df = fcen / 20
    o = vol(make, 1, [sz], 20, center_origin=True)
    o.add_pml(dpml)
    if upstream:
        o.set_upstream_nl(True)
    o.set_chi3(0, np.full(o.shape(), k))
    w = 1 / df
    o.add_gaussian_source(0, fcen, w, 0.0, 2 * w * 5.0, (0, 0, -0.5 * sz + dpml), 1.0)
    zf = 0.5 * sz - dpml - 0.5
    reg = [([0, 0, zf], [0, 0, zf], 2, 1.0)]
    h1 = o.add_dft_flux(reg, [fcen], 1)
    h3 = o.add_dft_flux(reg, [3 * fcen], 1)
    st, et = 0.0, 2 * w * 5.0  # last_source_time (src/meep.hpp:1024)
    peak, cut = 0.5 * (st + et), (et - st) * 0.5
    while math.exp(-cut * cut / (2 * w * w)) < 1e-100:
        cut *= 0.9
    ts = float(np.float32(peak + float(np.float32(cut))))
    clo = {"max_abs": 0, "cur_max": 0, "t0": 0}

    def stop():  # python/simulation.py:5250-5271
        v = o.get_field(0, (0, 0, zf))
        clo["cur_max"] = max(clo["cur_max"], abs(v) * abs(v))
        if o.round_time() <= 50 + clo["t0"]:
            return False
        old = clo["cur_max"]
        clo["cur_max"] = 0
        clo["t0"] = o.round_time()
        clo["max_abs"] = max(clo["max_abs"], old)
        return old <= clo["max_abs"] * decay

    while not (stop() and o.round_time() >= ts):
        o.step(1)
    return o, o.flux(h1)[0], o.flux(h3)[0]


# symmetric off-diagonal chi1inv pairs: value and region (inside the slab)
OFFD_PAIRS = {(0, 1): (0.04, lambda x, y, z: x < 0.3),
              (1, 2): (-0.03, lambda x, y, z: y > -0.4),
              (0, 2): (0.025, lambda x, y, z: z < 0.5)}


def sc_upstream_nl_3d(make, steps=50, lorentz=True, isrc=True, chi2=True, pml=True,
                      upstream=True, offdiag=False, chi3=True, scale=1.0):
    """Upstream-mode chi2 + chi3 slab (diagonal eps 2.25) crossing the PML boundary,
    a Lorentzian in part of it (D - P neighbour reads), an integrated source and a
    current source, strong fields (amp 40).  offdiag: symmetric off-diagonal
    chi1inv pairs, each in its own region (OFFD_PAIRS), so reference chunks keep
    both rows (3x3), one row (2x2, either order) or none."""
    o = vol(make, 3, [3.2, 3.2, 3.2], 10, center_origin=True)
    if pml:
        o.add_pml(0.8)
    if upstream:
        o.set_upstream_nl(True)
    sig = []
    for c in E_COMPS:
        x, y, z = o.coords(c)
        inside = np.abs(z - 0.2) < 0.9
        o.set_chi1inv(c, c, np.where(inside, 1 / 2.25, 1.0))
        if chi3:
            o.set_chi3(c, np.where(inside, 2e-2, 0.0))
        if offdiag:
            for k in (1, 2):
                d = (c + k) % 3
                val, reg = OFFD_PAIRS[tuple(sorted((c, d)))]
                o.set_chi1inv(c, d, np.where(inside & reg(x, y, z), val, 0.0))
        if chi2:
            o.set_chi2(c, np.where(inside & (x > -0.5), 3e-2, 0.0))
        sig.append(np.where(inside & (y > 0.2), 0.4, 0.0))
    if lorentz:
        o.add_lorentzian(1.3, 0.08, sig)
    o.add_gaussian_source(0, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, -0.3), 40.0 * scale)
    o.add_gaussian_source(1, 0.35, 4.0, 0.0, 40.0, (-0.4, 0.25, 0.35), 25.0 * scale,
                          is_integrated=isrc)
    o.step(steps)
    return o


def harmonics_cpp(make, chi2, chi3, J, upstream=True):
    """tests/harmonics.cpp:27-80 on the scenario interface: 1-D cell 110 @ res 20,
    PML 5, chi2 / chi3 everywhere, integrated Ex source gaussian_src_time(1/3,
    1/60) (C++ default: is_integrated) at z = -50, single-frequency DFT fluxes at
    f, 2f, 3f at z = 49.5; stepped until time() >= last_source_time(), then in
    50-unit rounds until the round's max |Ex| < 1e-6 of the overall max.
    Returns (sim, A2, A3) = (flux(2f) / flux(f), flux(3f) / flux(f))."""
    dpml, res, freq = 5.0, 20, 1.0 / 3.0
    sz = 100 + 2 * dpml
    o = vol(make, 1, [sz], res, center_origin=True)
    o.add_pml(dpml)
    if upstream:
        o.set_upstream_nl(True)
    o.set_chi2(0, np.full(o.shape(), chi2))
    o.set_chi3(0, np.full(o.shape(), chi3))
    w = 1.0 / (freq / 20)  # gaussian_src_time(f, fwidth, s = 5): peak = cutoff = 5 w
    o.add_gaussian_source(0, freq, w, 0.0, 10 * w, (0, 0, -0.5 * sz + dpml), J, is_integrated=True)
    zf = 0.5 * sz - dpml - 0.5
    hs = [o.add_dft_flux([([0, 0, zf], [0, 0, zf], 2, 1.0)], [k * freq], 1) for k in (1, 2, 3)]
    cut = 5 * w
    while math.exp(-cut * cut / (2 * w * w)) < 1e-100:
        cut *= 0.9
    last = float(np.float32(5 * w + float(np.float32(cut))))
    emax = 0.0
    while o.t * o.dt < last:
        emax = max(emax, abs(o.get_field(0, (0, 0, zf))))
        o.step(1)
    while True:
        emaxcur, T = 0.0, o.t * o.dt + 50
        while o.t * o.dt < T:
            e = abs(o.get_field(0, (0, 0, zf)))
            emax, emaxcur = max(emax, e), max(emaxcur, e)
            o.step(1)
        if emaxcur < 1e-6 * emax:
            break
    f1, f2, f3 = (o.flux(h)[0] for h in hs)
    return o, f2 / f1, f3 / f1


# ------------------------------------------------------------- conductivity
def sc_conductive_3d(make, steps=40, slabs_extra=None):
    """D and B conductivity (step_curl's cnd branches, src/step_generic.cpp:89-229):
    a conductive D slab x < 0.3 that reaches into the PML chunks on the low-x /
    y / z sides (f_cond chunks) but not the high-x ones, B conductivity in an
    interior box, a dielectric core, a current source inside the conductive
    slab (cndinv scaling, src/step.cpp:300-309) and an integrated one outside."""
    o = vol(make, 3, [3.2, 2.6, 3.0], 10, center_origin=True)
    o.add_pml(0.7)
    for c in E_COMPS:
        x, y, z = o.coords(c)
        o.set_chi1inv(c, c, np.where((np.abs(y) < 0.4) & (np.abs(z) < 0.4), 1 / 4.0, 1.0))
    for c in (6, 7, 8):  # Dx, Dy, Dz
        x, y, z = o.coords(c)
        o.set_conductivity(c, np.where(x < 0.3, 0.8 + 0.1 * (c - 6), 0.0))
    for c in (9, 10):  # Bx, By
        x, y, z = o.coords(c)
        box = (np.abs(x - 0.5) < 0.3) & (np.abs(y) < 0.5) & (np.abs(z) < 0.5)
        o.set_conductivity(c, np.where(box, 2.0, 0.0))
    o.add_gaussian_source(2, 0.3, 4.0, 0.0, 40.0, (-0.45, 0.05, 0.05), 1.0)
    o.add_gaussian_source(0, 0.25, 4.0, 0.0, 40.0, (0.75, -0.1, 0.2), 0.5, is_integrated=True)
    o.add_gaussian_source(3, 0.3, 4.0, 0.0, 40.0, (0.55, 0.1, 0.0), 0.7)  # Hx in the B box
    o.step(steps)
    return o


def pml1d_ft(make, res, sz, dpml, conductivity, freq=1.0, stretch=2.0, R=1e-15, max_steps=None):
    """One structure of tests/pml.cpp:check_pml1d (75-114): 1-D cell sz, pml(dpml, R,
    stretch), By conductivity everywhere, integrated Ex gaussian_src_time(freq,
    freq/20) at -sz/2 + dpml_0 + 0.1 (dpml_0 = 1), and do_ft (49-73): the Fourier
    transform of Ex at sz/2 - dpml_0 - 0.1 summed over every step until the fields
    have decayed.  Returns (ft, steps)."""
    o = make(1, [0, 0, int(sz * res + 0.5)], res, 0.5, [0, 0, -int(sz * res + 0.5)])
    o.add_pml(dpml, R=R, mean_stretch=stretch)
    o.set_conductivity(10, np.full(o.shape(), float(conductivity)))  # By
    width = 1.0 / (freq / 20)
    o.add_gaussian_source(0, freq, width, 0.0, 2 * width * 5.0, (0, 0, -0.5 * 3.0 + 1.0 + 0.1),
                          1.0, is_integrated=True)
    last = float(np.float32(width * 5.0 + width * 5.0))
    pt = (0, 0, 0.5 * 3.0 - 1.0 - 0.1)
    ft = 0j
    emax = 0.0
    n = 0

    def sample():
        nonlocal ft, emax
        v = o.get_field(0, pt)
        ft += v * complex(math.cos(2 * math.pi * freq * o.time()),
                          math.sin(2 * math.pi * freq * o.time()))
        return abs(v)

    while o.time() < last:
        emax = max(emax, sample())
        o.step()
        n += 1
    while True:
        emaxcur = 0.0
        T = o.time() + 50
        while o.time() < T:
            e = sample()
            emax = max(emax, e)
            emaxcur = max(emaxcur, e)
            o.step()
            n += 1
            if max_steps and n >= max_steps:
                return ft, n
        if emaxcur < 1e-6 * emax:
            break
        if T > 500 and emaxcur > 1e-2 * emax:
            raise RuntimeError("meep: fields do not seem to be decaying")
    return ft, n


def check_pml1d(make, conductivity=10.0, nres=8):
    """tests/pml.cpp:check_pml1d (75-114, run by main at 323 with conductivity 10):
    the reflection |ft - ft2|^2/|ft2|^2 against a cell with twice the PML must fall
    at least as fast as ((res-10)/res)^8 * 1.1 from one resolution to the next.
    Returns the list of (res, refl) and whether the reference's check passes."""
    dpml = 1.0
    sz, sz2 = 1.0 + 2 * dpml, 1.0 + 2 * dpml * 2
    out, ok, prev = [], True, 0.0
    for i in range(nres):
        res = 10.0 + 10.0 * i
        ft, _ = pml1d_ft(make, res, sz, dpml, conductivity)
        ft2, _ = pml1d_ft(make, res, sz2, 2 * dpml, conductivity)
        refl = abs(ft - ft2) ** 2 / abs(ft2) ** 2
        out.append((res, refl))
        if i > 0 and refl > prev * ((res - 10) / res) ** 8 * 1.1:
            ok = False
        prev = refl
    return out, ok


def sc_conductive_2d(make, steps=80):
    """2-D TE + TM with conductivity on every D / B component across a one-sided PML."""
    o = vol(make, 2, [2.3, 1.9], 10)
    o.add_pml(0.5, dirs=(0,), sides=(1,))
    o.add_pml(0.4, dirs=(1,), sides=(0,))
    for c in range(6, 12):
        x, y = o.coords(c)
        o.set_conductivity(c, np.where(x > 1.0, 0.3 + 0.05 * c, 0.0))
    o.add_gaussian_source(5, 0.4, 3.0, 0.0, 30.0, (1.03, 0.77), 2.0)
    o.add_gaussian_source(2, 0.35, 3.0, 0.0, 30.0, (1.4, 1.1), 1.0)
    o.step(steps)
    return o


# ------------------------------------------------- anisotropic Lorentzian
def sc_aniso_lorentz_3d(make, steps=40, full=True):
    """Anisotropic Lorentzian sigma (update_P's 3x3 / 2x2 branches and OFFDIAG
    averaging, src/susceptibility.cpp:185-250): a slab with a full symmetric
    tensor crossing into the PML chunks (f_w as W), a second susceptibility with
    only an xy term in a box (2x2 branch; isotropic chunks elsewhere), eps."""
    o = vol(make, 3, [3.2, 2.8, 3.0], 10, center_origin=True)
    o.add_pml(0.7)
    for c in E_COMPS:
        x, y, z = o.coords(c)
        o.set_chi1inv(c, c, np.where(np.abs(z) < 0.6, 1 / 2.25, 1.0))
    diag = (0.5, 0.4, 0.3)
    off = {(0, 1): 0.12, (0, 2): 0.07, (1, 2): 0.05} if full else {(0, 1): 0.12}
    sig = [[None] * 3 for _ in range(3)]
    for c in E_COMPS:
        x, y, z = o.coords(c)
        sig[c][c] = np.where(np.abs(z) < 0.6, diag[c], 0.0)
        h = 0.5 / 10  # off-diagonal entries half a pixel back along c
        xs, ys, zs = x - h * (c == 0), y - h * (c == 1), z - h * (c == 2)
        for (a, b), v in off.items():
            for (r, col) in ((a, b), (b, a)):
                if r == c:
                    sig[c][col] = np.where(np.abs(zs) < 0.6, v, 0.0)
    o.add_lorentzian_tensor(1.1, 0.05, sig)
    sig2 = [[None] * 3 for _ in range(3)]
    for c in E_COMPS:
        x, y, z = o.coords(c)
        box = (np.abs(x - 0.3) < 0.5) & (np.abs(y) < 0.4) & (z > 0.7) & (z < 1.2)
        sig2[c][c] = np.where(box, 0.3, 0.0)
        if c in (0, 1):
            sig2[c][1 - c] = np.where(box, 0.1, 0.0)
    o.add_lorentzian_tensor(0.8, 0.1, sig2)
    o.add_gaussian_source(0, 0.3, 4.0, 0.0, 40.0, (0.05, 0.05, -0.2), 10.0)
    o.add_gaussian_source(1, 0.35, 4.0, 0.0, 40.0, (0.4, -0.1, 0.9), 5.0)
    o.step(steps)
    return o


# --------------------------------------------------------- custom sources
def _chirp(t):
    return complex(math.exp(-((t - 4.0) / 1.5) ** 2) * math.cos(2 * math.pi * 0.3 * t * (1 + 0.05 * t)),
                   0.1 * math.sin(0.7 * t))


def sc_custom_source_3d(make, steps=50):
    """custom_src_time (src/meep.hpp:1059-1092): a chirped current source, the same
    function again at another point (merged src_time), an integrated custom
    source, with PML and a dielectric core."""
    o = vol(make, 3, [3.0, 2.6, 2.2], 10, center_origin=True)
    o.add_pml(0.6)
    for c in E_COMPS:
        x, y, z = o.coords(c)
        o.set_chi1inv(c, c, np.where(np.abs(y) < 0.4, 0.25, 1.0))
    o.add_custom_source(2, _chirp, 0.0, 9.0, (0.05, 0.02, 0.01), 1.0)
    o.add_custom_source(2, _chirp, 0.0, 9.0, (-0.43, 0.31, 0.2), complex(0.3, 0.4))
    o.add_custom_source(0, lambda t: math.sin(0.9 * t) * math.exp(-0.1 * t), 0.5, 7.3,
                        (0.2, -0.3, -0.1), 0.8, is_integrated=True)
    o.step(steps)
    return o


# subpixel-averaged structure (mnl_structure_set_epsilon_geometry): a core along x,
# a sphere overriding it, cylinders along z and x
OBJS_3D = [
    [0, 6.0, 0.0, 0.0, 0.0, 1e20, 0.43, 0.37],           # waveguide core along x
    [1, 11.0, 0.121, -0.087, 0.053, 0.52, 0.0, 0.0],      # sphere (overrides the core)
    [2, 2.5, -0.31, 0.27, 0.0, 0.18, 0.9, 2.0],           # cylinder along z
    [2, 3.5, 0.0, 0.33, -0.29, 0.15, 1.1, 0.0],           # cylinder along x
]


def sc_averaged(make, upstream=False, steps=30):
    o = vol(make, 3, [3.0, 2.8, 3.2], 10, center_origin=True)
    o.add_pml(0.6)
    o.set_epsilon_geometry(OBJS_3D, 1.7)
    if upstream:
        o.set_upstream_nl(True)
        for c in range(3):
            x, y, z = o.coords(c)
            o.set_chi3(c, np.where(np.abs(z) < 0.5, 1e-2, 0.0))
    o.add_gaussian_source(2, 0.3, 3.0, 0.0, 30.0, (0.05, 0.05, 0.05), 1.0)
    o.add_gaussian_source(0, 0.35, 3.0, 0.0, 30.0, (-0.2, 0.1, -0.3), 0.7)
    o.step(steps)
    return o


def sc_c4_nr(make, steps=25, n=256):
    """BASELINE configs[3] NR sub-variant at full size (bench.py --workload kerr_nr):
    Kerr chi3 + Lorentzian slab |z| <= 2 (eps 2.25), chi2 0.5 in the box |x|,|y| <= 3,
    |z| <= 1.5 with chi1inv off-diagonal 1e-3 strictly inside it (the Newton-Raphson E
    update), PML(1.0), Ex Gaussian at z = -3 with amplitude 50, fields from zero.  Its
    strong fields make some voxels' first NR attempts fail (random-seed fallbacks
    included), which exercises the deferred parallel-attempt pass."""
    L = n / 10.0
    o = vol(make, 3, [L, L, L], 10, center_origin=True)
    o.add_pml(1.0)
    sig = []
    for c in E_COMPS:
        x, y, z = o.coords(c)
        slab = np.abs(z) <= 2.0
        o.set_chi1inv(c, c, np.where(slab, 1 / 2.25, 1.0))
        o.set_chi3(c, np.where(slab, 1e-2, 0.0))
        sig.append(np.where(slab, 0.5, 0.0))
        box = (np.abs(x) <= 3.0) & (np.abs(y) <= 3.0) & (np.abs(z) <= 1.5)
        o.set_chi2(c, np.where(box, 0.5, 0.0))
        inner = (np.abs(x) < 3.0) & (np.abs(y) < 3.0) & (np.abs(z) < 1.5)
        off = np.where(inner, 1e-3, 0.0)
        for d in range(3):
            if d != c:
                o.set_chi1inv(c, d, off)
        del x, y, z, slab, box, inner, off
    o.add_lorentzian(1.1, 0.05, sig)
    o.add_gaussian_source(0, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, -3.0), 50.0)
    o.step(steps)
    return o


# ------------------------------------------------------------------ H-side materials
# mu != 1 (chi1inv of the H components, structure::set_mu) and magnetic Lorentzian
# susceptibilities (update_eh(H_stuff) + update_pols(H_stuff), src/step.cpp:75-92,
# src/update_eh.cpp:67-283): DESIGN.md section 23.

def _box_fn(lo, hi, inside, outside=1.0):
    def fn(*p):
        m = np.ones_like(p[0], dtype=bool)
        for k, x in enumerate(p):
            m &= (x > lo[k]) & (x < hi[k])
        return np.where(m, inside, outside)
    return fn


def sc_mu_1d(make, steps=300, lorentz=False):
    """1-D: a mu = 3 slab inside the cell, PML at both ends, Ex Gaussian current."""
    o = vol(make, 1, [12.0], 10, center_origin=True)
    o.add_pml(1.0)
    o.set_mu_fn(_box_fn((-1.5,), (2.0,), 3.0))
    if lorentz:  # magnetic Drude-Lorentz slab overlapping the mu slab
        z = o.coords(4)[-1]
        o.add_magnetic_lorentzian(1.1, 0.05, [None, np.where(np.abs(z - 1.0) < 1.5, 0.5, 0.0), None])
    o.add_gaussian_source(0, 0.3, 3.0, 0.0, 30.0, (0, 0, -3.0), 1.0)
    o.step(steps)
    return o


def sc_mu_2d(make, te=True, steps=120, lorentz=False):
    """2-D TE (Hz source) or TM (Ez source): an anisotropic (diagonal) mu block that
    crosses the one-sided PML chunk boundary, odd grid."""
    o = vol(make, 2, [3.1, 2.7], 10)
    o.add_pml(0.5, dirs=(0,), sides=(1,))
    o.add_pml(0.4, dirs=(1,), sides=(0,))
    for c, m in ((3, 2.0), (4, 1.5), (5, 3.0)):
        o.set_chi1inv(c, c % 3, 1.0 / _box_fn((1.0, 0.2), (3.0, 1.6), m)(*o.coords(c)))
    if lorentz:
        sig = []
        for c in (3, 4, 5):
            sig.append(_box_fn((0.5, 0.9), (2.0, 2.2), 0.4, 0.0)(*o.coords(c)))
        o.add_magnetic_lorentzian(0.8, 0.1, sig)
    if te:
        o.add_gaussian_source(5, 0.4, 3.0, 0.0, 30.0, (1.03, 0.77), 2.0)
    else:
        o.add_gaussian_source(2, 0.4, 3.0, 0.0, 30.0, (1.03, 0.77), 2.0)
    o.step(steps)
    return o


def sc_mu_3d(make, steps=40, lorentz=False, offdiag=False, eps=True, sizes=(3.2, 3.0, 3.4)):
    """3-D with PML: a mu block crossing PML chunks (diagonal mu 2 / 3 / 1.5), an eps
    waveguide, optionally a magnetic Lorentzian box and an off-diagonal mu row confined
    to the +x PML chunk (inert in the fork's H update, but it keeps H separate there)."""
    o = vol(make, 3, list(sizes), 10, center_origin=True)
    o.add_pml(0.7)
    lo, hi = (-0.6, -0.9, -2.0), (1.2, 0.5, 0.3)
    for c, m in ((3, 2.0), (4, 3.0), (5, 1.5)):
        o.set_chi1inv(c, c % 3, 1.0 / _box_fn(lo, hi, m)(*o.coords(c)))
    if offdiag:
        x, y, z = o.coords(4)
        o.set_chi1inv(4, 0, np.where(x > 1.05, 1e-3, 0.0))
    if eps:
        for c in (0, 1, 2):
            o.set_chi1inv(c, c, 1.0 / _box_fn((-9, -0.4, -0.3), (9, 0.4, 0.3), 6.0)(*o.coords(c)))
    if lorentz:
        sig = [_box_fn((-0.8, -0.5, -0.6), (0.6, 1.3, 1.5), 0.6, 0.0)(*o.coords(c)) for c in (3, 4, 5)]
        o.add_magnetic_lorentzian(0.9, 0.08, sig)
        o.add_magnetic_lorentzian(1.0, 0.2, [None, sig[1] * 0.5, None], drude=True)
    o.add_gaussian_source(2, 0.3, 3.0, 0.0, 30.0, (0.05, -0.15, 0.1), 1.0)
    o.add_gaussian_source(4, 0.35, 3.0, 0.0, 30.0, (-0.3, 0.2, -0.4), 0.5)
    o.step(steps)
    return o
