"""GPU parity: HIP product path vs the CPU oracle on identical inputs.

Tolerance: the product is compiled with -ffp-contract=off and follows the
reference's expression order, so arrays are required to be BITWISE equal
(max |diff| == 0).  Golden reference values (tests/golden) are required bit
for bit as well, except known_results (rel 1e-5 as in the reference test).
"""
import math

import numpy as np
import pytest

from scenarios import (ALL_COMPS, ProductSim, compare_all, make_oracle, sc_big_box_3d, sc_cfg1,
                       sc_kerr_lorentz_3d, sc_known_metallic_3d, sc_known_pml_2d,
                       sc_multi_source_3d, sc_nr_pml_dispersive, sc_nr_probe, sc_polariton_1d,
                       sc_te_magnetic_2d, sc_vacuum_pml_3d, sc_waveguide_3d)

pytestmark = pytest.mark.gpu


def _bitwise(prod, orc, comps=ALL_COMPS):
    diffs = compare_all(prod, orc, comps)
    bad = {c: d for c, d in diffs.items() if d != 0.0}
    assert not bad, f"max|diff| per component: {bad}"


def test_cfg1_golden_and_arrays(golden):
    g = golden["survey_cfg1"]
    p = sc_cfg1(ProductSim)
    assert p.get_field(2, (0.5, 0.3)) == g["ez_0p5_0p3"]
    assert p.get_field(2, (0.0, 0.0)) == g["ez_0_0"]
    ss = 0.0
    for ix in range(-95, 96, 5):
        for iy in range(-95, 96, 5):
            v = p.get_field(2, (ix * 0.1, iy * 0.1))
            ss += v * v
    assert ss == g["sumsq_39x39"]
    o = sc_cfg1(make_oracle, steps=500)
    _bitwise(p, o, comps=(2, 3, 4, 8, 9, 10))


def test_vacuum_pml_3d():
    _bitwise(sc_vacuum_pml_3d(ProductSim), sc_vacuum_pml_3d(make_oracle))


def test_waveguide_3d():
    _bitwise(sc_waveguide_3d(ProductSim), sc_waveguide_3d(make_oracle))


def test_kerr_lorentz_3d():
    _bitwise(sc_kerr_lorentz_3d(ProductSim), sc_kerr_lorentz_3d(make_oracle))


def test_nr_probe_golden(golden):
    g = golden["survey_nr"]
    for c2, key in ((0.0, "ex_chi2_0"), (0.5, "ex_chi2_0p5")):
        p = sc_nr_probe(ProductSim, c2)
        cen = p.center()
        v = p.get_field(0, [cen[0] + 0.21, cen[1] + 0.13, cen[2] + 0.07])
        assert v == g[key]
        assert p.nr_random_fallbacks() == 0
        _bitwise(p, sc_nr_probe(make_oracle, c2))


def test_nr_pml_dispersive():
    _bitwise(sc_nr_pml_dispersive(ProductSim), sc_nr_pml_dispersive(make_oracle))


def test_nr_integrated_source_on_chunk_seam():
    """Integrated sources on a reference chunk seam next to chi2 NR voxels: the
    dipole is subtracted only by readers in the owning chunk (the reference's
    per-chunk f_minus_p, src/update_eh.cpp:136-146)."""
    from scenarios import sc_nr_isrc_seam
    p = sc_nr_isrc_seam(ProductSim)
    assert p.nr_random_fallbacks() == 0
    _bitwise(p, sc_nr_isrc_seam(make_oracle))


def test_nr_chi2_from_boxes():
    """chi2 given as a device-rasterised box (mnl_structure_set_box kind 1, the
    bench's fast setup) enables the Newton-Raphson branch exactly as the same
    chi2 given as an array (points with lo <= pos <= hi, no averaging)."""
    box = (-0.5, 0.5, -0.45, 0.55, -0.5, 0.3)

    def run(make, use_box):
        o = make(3, [26, 26, 26], 10.0, 0.5, [-26, -26, -26])
        o.add_pml(0.6)
        for c in range(3):
            x, y, z = o.coords(c)
            inside = ((x >= box[0]) & (x <= box[1]) & (y >= box[2]) & (y <= box[3]) &
                      (z >= box[4]) & (z <= box[5]))
            for d in range(3):
                o.set_chi1inv(c, d, np.where(inside, 0.25 if d == c else 1e-3, 1.0 if d == c else 0.0))
            if not use_box:
                o.set_chi2(c, np.where(inside, 0.5, 0.0))
        if use_box:
            o.s.set_box(1, list(box), 0.5)
        o.legacy_point_source(2, 0.5, 0.5, 0.0, 3.0, (0.05, 0.05, 0.05), 5.0)
        o.step(30)
        return o
    p = run(ProductSim, True)
    assert not p._fields().fused_active()  # NR keeps the step unfused
    _bitwise(p, run(make_oracle, False))


def test_known_results(golden):
    kr = golden["known_results"]
    p = sc_known_metallic_3d(ProductSim)
    v = p.get_field(2, p.center())
    assert abs(v - kr["metallic_3d_ez"]) < abs(kr["metallic_3d_ez"]) * kr["rel_tol"]
    p = sc_known_pml_2d(ProductSim)
    v = p.get_field(2, p.center())
    assert abs(v - kr["pml_2d_tm_ez"]) < abs(kr["pml_2d_tm_ez"]) * kr["rel_tol"]
    _bitwise(p, sc_known_pml_2d(make_oracle), comps=(2, 3, 4, 8, 9, 10))


def test_polariton_1d(golden):
    kr = golden["known_results"]
    p = sc_polariton_1d(ProductSim)
    v = p.get_field(0, p.center())
    assert abs(v - kr["polariton_1d_ex"]) < abs(kr["polariton_1d_ex"]) * kr["rel_tol"]
    _bitwise(p, sc_polariton_1d(make_oracle), comps=(0, 4, 6, 10))


def test_te_magnetic_2d():
    _bitwise(sc_te_magnetic_2d(ProductSim), sc_te_magnetic_2d(make_oracle),
             comps=(0, 1, 5, 6, 7, 11))


def test_multi_source_3d():
    _bitwise(sc_multi_source_3d(ProductSim), sc_multi_source_3d(make_oracle))


def test_simulation_api_matches_core():
    import meep_nl_amd as mp
    sim = mp.Simulation(cell_size=mp.Vector3(2.0, 2.0, 0), resolution=10,
                        sources=[mp.Source(mp.GaussianSource(0.15, fwidth=0.1), mp.Ez,
                                           center=mp.Vector3())])
    sim.run(until=5.0)
    p = ProductSim(2, [20, 20, 0], 10, 0.5, [-20, -20, 0])
    p.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0, 0), 1.0)
    p.step(sim.timestep)
    np.testing.assert_array_equal(sim.get_component_array(mp.Ez), p.get_array(2))
    assert sim.meep_time() == pytest.approx(sim.timestep * 0.05)


@pytest.mark.parametrize("zchunk", ["64", "7"])
def test_fused_many_tiles(monkeypatch, zchunk):
    """The fused interior kernel over many (x,y) tiles and z-chunks (zchunk 7 puts a
    chunk seam every 7 planes) must stay bitwise equal to the oracle."""
    monkeypatch.setenv("MNL_FUSED_ZCHUNK", zchunk)
    p = sc_big_box_3d(ProductSim)
    assert p._fields().kernel_stats(0)[0] >= 0
    _bitwise(p, sc_big_box_3d(make_oracle))


def test_fused_vs_unfused(monkeypatch):
    monkeypatch.setenv("MNL_NO_FUSED", "1")
    a = sc_big_box_3d(ProductSim, steps=16)
    monkeypatch.delenv("MNL_NO_FUSED")
    b = sc_big_box_3d(ProductSim, steps=16)
    _bitwise(a, b)


def test_fused_mode_toggle():
    """Adding a magnetic (non-fusable) source mid-run switches the fused interior
    off (E is materialised from D) and the run continues bitwise."""
    def add_h(o):
        o.add_gaussian_source(4, 0.3, 3.0, 0.0, 30.0, (1.0, 0.3, -1.1), 0.8)
    _bitwise(sc_big_box_3d(ProductSim, steps=24, extra=add_h),
             sc_big_box_3d(make_oracle, steps=24, extra=add_h))


def test_fused_palette_used():
    """Two distinct chi1inv values: the fused kernel reads them through the byte
    palette (4 B/cell instead of 24) and stays bitwise equal to the oracle."""
    p = sc_big_box_3d(ProductSim, steps=12)
    f = p._fields()
    assert f.fused_active() and f.fused_palette()
    _bitwise(p, sc_big_box_3d(make_oracle, steps=12))


def test_fused_f64_chi1inv(monkeypatch):
    monkeypatch.setenv("MNL_NO_PALETTE", "1")
    p = sc_big_box_3d(ProductSim, steps=12)
    assert p._fields().fused_active() and not p._fields().fused_palette()
    _bitwise(p, sc_big_box_3d(make_oracle, steps=12))


def test_fused_many_distinct_chi1inv():
    """More distinct chi1inv values than the palette holds: f64 chi1inv path."""
    p = sc_big_box_3d(ProductSim, steps=12, random_eps=True)
    assert p._fields().fused_active() and not p._fields().fused_palette()
    _bitwise(p, sc_big_box_3d(make_oracle, steps=12, random_eps=True))


@pytest.mark.parametrize("dist", ["1", "2"])
def test_fused_prefetch_distance(monkeypatch, dist):
    monkeypatch.setenv("MNL_FUSED_DIST", dist)
    _bitwise(sc_big_box_3d(ProductSim, steps=10), sc_big_box_3d(make_oracle, steps=10))


def test_fused_lorentz_big_box():
    """Lorentzian slab inside a big box: fused step with the polarization box in the
    general kernels and lean tiles around it, bitwise."""
    from scenarios import sc_big_lorentz_3d
    p = sc_big_lorentz_3d(ProductSim)
    assert p._fields().fused_active()
    _bitwise(p, sc_big_lorentz_3d(make_oracle))


def test_fused_lorentz_toggle():
    """Leaving fused mode inside the polarization box materialises W_E from Pprev."""
    from scenarios import sc_big_lorentz_3d

    def add_h(o):
        o.add_gaussian_source(4, 0.3, 3.0, 0.0, 30.0, (1.0, 0.3, 2.2), 0.8)
    _bitwise(sc_big_lorentz_3d(ProductSim, extra=add_h),
             sc_big_lorentz_3d(make_oracle, extra=add_h))


@pytest.mark.parametrize("freq,width,end", [(0.35, 10.0, 40.0), (0.35, 4.0, 100.0), (0.27, 3.0, 30.0)])
def test_source_values_bitwise(freq, width, end):
    """Per-step source amplitudes are computed on the host with libgcc's complex
    arithmetic (__divdc3 / __muldc3, like the reference and the oracle): the
    library is linked with g++ so clang's compiler-rt versions, which round
    1/(-2*pi*f*i) differently for some f, are not pulled in."""
    from scenarios import vol
    res = []
    for make in (ProductSim, make_oracle):
        o = vol(make, 3, [1.6, 1.6, 1.6], 10, center_origin=True)
        o.add_gaussian_source(2, freq, width, 0.0, end, (0.05, 0.05, 0.05), 1.0)
        o.add_continuous_source(0, freq * 1.1, 2.0, 0.0, 1e20, 3.0, (-0.25, 0.15, 0.05), 0.5)
        o.step(6)
        res.append(o)
    _bitwise(*res)


@pytest.mark.parametrize("G", ["product", "slabs3"])
def test_nr_lorentz_on_metal_walls(G):
    """Newton-Raphson E and a Lorentzian reaching the metallic walls: E is updated
    on the high wall planes the reference's chunks own (D = 0 there, nonzero
    through the NR neighbour reads), update_P keeps that transient, then the walls
    are zeroed; across slab seams only the owning chunk sees the wall P."""
    from scenarios import GroupSim3, sc_nr_wall_lorentz
    make = ProductSim if G == "product" else GroupSim3
    p = sc_nr_wall_lorentz(make)
    o = sc_nr_wall_lorentz(make_oracle)
    assert float(np.max(np.abs(o.get_array(2)))) > 0
    assert o.nr_random_fallbacks() == 0  # no random restarts: the streams differ
    _bitwise(p, o)
