"""H-side materials on the GPU: mu != 1 (chi1inv of the H
components, update_eh(H_stuff) -> step_update_EDHB, src/update_eh.cpp:67-283,
src/step_generic.cpp:576-906) and magnetic Lorentzian susceptibilities
(update_pols(H_stuff), src/step.cpp:75-92), bitwise against the oracle in 1-D, 2-D TE
and TM, 3-D with PML on one GPU and 2 / 3 slabs; monitors that read H and B (DFT
flux and fields, energies with the synchronized magnetic fields, slices of B across
chunk seams), checkpoints and initialize_field."""
import os

import numpy as np
import pytest

from scenarios import (ALL_COMPS, GroupSim, GroupSim3, ProductSim, compare_all, flux_box_faces,
                       make_oracle, random_init, sc_mu_1d, sc_mu_2d, sc_mu_3d)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _bitwise(p, o, comps=ALL_COMPS):
    d = {c: v for c, v in compare_all(p, o, comps).items() if v != 0.0}
    assert not d, d


@pytest.mark.parametrize("lorentz", [False, True])
def test_mu_1d(lorentz):
    _bitwise(sc_mu_1d(ProductSim, lorentz=lorentz), sc_mu_1d(make_oracle, lorentz=lorentz),
             (0, 4, 6, 10))


@pytest.mark.parametrize("te", [True, False])
@pytest.mark.parametrize("lorentz", [False, True])
def test_mu_2d(te, lorentz):
    comps = (0, 1, 5, 6, 7, 11) if te else (2, 3, 4, 8, 9, 10)
    _bitwise(sc_mu_2d(ProductSim, te=te, lorentz=lorentz),
             sc_mu_2d(make_oracle, te=te, lorentz=lorentz), comps)


@pytest.mark.parametrize("G", [ProductSim, GroupSim, GroupSim3])
@pytest.mark.parametrize("lorentz,offdiag", [(False, False), (True, False), (True, True)])
def test_mu_3d(G, lorentz, offdiag):
    _bitwise(sc_mu_3d(G, lorentz=lorentz, offdiag=offdiag),
             sc_mu_3d(make_oracle, lorentz=lorentz, offdiag=offdiag))


def test_mu_3d_no_eps_fused_off():
    """mu only (no eps, vacuum otherwise): the fused step is off, results bitwise."""
    p = sc_mu_3d(ProductSim, eps=False)
    assert not p.f.fused_active()
    _bitwise(p, sc_mu_3d(make_oracle, eps=False))


FREQS = [0.25, 0.3, 0.35]


def _monitors(make, lorentz):
    o = sc_mu_3d(make, steps=0, lorentz=lorentz, offdiag=True)
    hs = [o.add_dft_flux(flux_box_faces([-0.42, -0.37, -0.33], [0.44, 0.51, 0.38], 3), FREQS, 1),
          o.add_dft_flux([([0.83, -1.5, -1.7], [0.83, 1.5, 1.7], 0, 1.0)], FREQS, 1)]
    df = o.add_dft_fields([3, 4, 5], [-1.3, -1.2, -1.4], [1.1, 0.9, 1.0], FREQS, False, 1)
    o.step(30)
    return o, hs, df


@pytest.mark.parametrize("G", [ProductSim, GroupSim3])
@pytest.mark.parametrize("lorentz", [False, True])
def test_mu_monitors(G, lorentz):
    p, hp, dp = _monitors(G, lorentz)
    o, ho, do = _monitors(make_oracle, lorentz)
    rtol = 0.0 if G is ProductSim else 1e-12  # slabs: per-rank partial sums
    for a, b in zip(hp, ho):
        fp, fo = np.asarray(p.flux(a)), np.asarray(o.flux(b))
        assert np.allclose(fp, fo, rtol=rtol, atol=0.0), (fp, fo)
        if G is ProductSim:
            for which in (0, 1):
                assert np.array_equal(p.dft_data(a, which), o.dft_data(b, which))
    for c in (3, 4, 5):
        for k in range(len(FREQS)):
            assert np.array_equal(p.dft_array(dp, c, k), o.dft_array(do, c, k)), (c, k)
    for name in ("electric_energy_in_box", "magnetic_energy_in_box", "field_energy_in_box"):
        ep, eo = getattr(p, name)(), getattr(o, name)()
        assert abs(ep - eo) <= 1e-12 * abs(eo), (name, ep, eo)
    vols = [([-1.6, -1.5, -1.7], [1.6, 1.5, 1.7]), ([-1.3, -0.2, 0.55], [0.4, 1.1, 0.55]),
            ([-0.3, 0.2, -0.55], [0.3, 0.2, 0.62]), ([0.9, -1.5, -1.7], [0.9, 1.5, 1.7])]
    for c in (3, 4, 5, 9, 10, 11):
        for lo, hi in vols:
            a, b = p.get_array_slice(c, lo, hi), o.get_array_slice(c, lo, hi)
            assert np.array_equal(a, b), (c, lo, hi, float(np.max(np.abs(a - b))))


@pytest.mark.parametrize("G", [ProductSim, GroupSim3])
def test_mu_checkpoint(G, tmp_path):
    path = os.path.join(str(tmp_path), "mu.mnl")
    a = sc_mu_3d(G, steps=0, lorentz=True, offdiag=True)
    a.step(13)
    a.dump(path)
    a.step(11)
    b = sc_mu_3d(G, steps=0, lorentz=True, offdiag=True)
    b.load(path)
    b.step(11)
    _bitwise(a, b)


@pytest.mark.parametrize("G", [ProductSim, GroupSim])
def test_mu_initialize_field(G):
    """Random B, H and D everywhere (every chunk, seam and wall) on a mu + magnetic
    Lorentzian structure, then stepping: the lazily separated H (a copy of B at the
    first H update) and the H copy of aliasing chunks follow the reference."""
    def run(make):
        o = sc_mu_3d(make, steps=0, lorentz=True, offdiag=True, sizes=(2.4, 2.2, 2.6))
        random_init(o, (9, 10, 11, 3, 7), seed=11)
        o.step(15)
        return o
    _bitwise(run(G), run(make_oracle))


def test_simulation_mu_and_magnetic_lorentzian():
    """meep.Simulation with Medium(mu=..., H_susceptibilities=[...]) (no averaging):
    the structure it builds, stepped, equals the oracle given the same per-point mu and
    sigma (Block.contains at the H Yee points)."""
    import meep_nl_amd as mp
    import scenarios as S
    blk = mp.Block(center=mp.Vector3(0.2, -0.1), size=mp.Vector3(1.2, 0.8),
                   material=mp.Medium(epsilon=2.0, mu=2.5, H_susceptibilities=[
                       mp.LorentzianSusceptibility(frequency=0.9, gamma=0.1, sigma=0.4)]))
    sim = mp.Simulation(cell_size=mp.Vector3(3.0, 2.6), resolution=10, geometry=[blk],
                        boundary_layers=[mp.PML(0.5)], eps_averaging=False,
                        sources=[mp.Source(mp.GaussianSource(0.3, fwidth=0.2), mp.Ez,
                                           center=mp.Vector3(0.05, 0.05))])
    assert sim.has_mu()
    sim.run(until=3.0)
    o = S.vol(make_oracle, 2, [3.0, 2.6], 10, center_origin=True)
    o.add_pml(0.5)

    def inside(c):
        x, y = o.coords(c)
        return blk.contains(x, y, np.zeros_like(x))
    o.set_chi1inv(2, 2, np.where(inside(2), 0.5, 1.0))
    for c in (0, 1):
        o.set_chi1inv(c, c, np.where(inside(c), 0.5, 1.0))
    for c in (3, 4, 5):
        o.set_chi1inv(c, c % 3, np.where(inside(c), 1 / 2.5, 1.0))
    o.add_magnetic_lorentzian(0.9, 0.1, [np.where(inside(c), 0.4, 0.0) for c in (3, 4, 5)])
    o.add_gaussian_source(2, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05), 1.0)
    o.step(sim.timestep)
    for c in (2, 3, 4, 8, 9, 10):
        assert sim.get_component_array(c).tobytes() == o.get_array(c).tobytes(), c
