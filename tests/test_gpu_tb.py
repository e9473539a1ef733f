"""Temporal blocking: pairs of fields::step() (src/step.cpp:35-140)
as rim (one-step tile kernel) + L2 (two-step kernel) + rim must be bit for bit the
one-step path and the CPU oracle.

Grids are large enough for a non-empty L2 (the lean box shrunk by 2, x aligned) and carry
seeded random D / B everywhere (initialize_field), so every two-step item, rim item, hole
around a source point and border face holds data from the first step."""
import os

import numpy as np
import pytest

from scenarios import ALL_COMPS, GroupSim, GroupSim3, ProductSim, make_oracle, random_init, vol

pytestmark = pytest.mark.gpu

E_COMPS = (0, 1, 2)
SRCS = ((0.37, -0.21, 0.05), (-3.3, 1.6, 2.15), (2.1, 0.3, -2.9), (0.4, -0.2, 0.1))


def sc_tb(make, sizes=(9.6, 6.4, 8.0), dpml=0.7, eps=6.0, random_eps=False, srcs=SRCS,
          steps=(1, 10), tb=True, rand=True, profile=False, schedule=()):
    """Dielectric slab across the PML boundary, Gaussian currents inside L2 (holes), near
    its edge and inside the PML; random initial fields; stepped in the given calls."""
    o = vol(make, 3, list(sizes), 10, center_origin=True)
    o.add_pml(dpml)
    if eps:
        for c in E_COMPS:
            x, y, z = o.coords(c)
            inside = (np.abs(y) < 0.8) & (z > -0.4) & (z < 3.0)
            if random_eps:
                val = 1.0 / np.random.default_rng(99 + c).uniform(1.0, 12.0, size=x.shape)
            else:
                val = 1.0 / eps
            o.set_chi1inv(c, c, np.where(inside, val, 1.0))
    for i, p in enumerate(srcs):
        o.add_gaussian_source(i % 3, 0.25, 4.0, 0.0, 40.0, p, 1.0 - 0.1 * i)
    if rand:
        random_init(o, (6, 7, 8, 9, 10, 11))
    if isinstance(o, ProductSim):
        for f in (o._all() if hasattr(o, "_all") else [o._fields()]):
            f.set_temporal_blocking(tb)
            for opt, val in schedule:  # Fields.set_schedule: same arithmetic, other schedule
                f.set_schedule(opt, val)
            if profile:
                f.set_profiling(True)
    for n in steps:
        o.step(n)
    return o


def _same(a, b):
    """Bitwise equality of all twelve components; on failure, per component the largest
    difference, the number of differing points and their index bounding box."""
    bad = {}
    for c in ALL_COMPS:
        x, y = a.get_array(c), b.get_array(c)
        neq = (x != y) & ~(np.isnan(x) & np.isnan(y))
        if neq.any():
            idx = np.argwhere(neq)
            bad[c] = (float(np.nanmax(np.abs(x - y))), int(neq.sum()),
                      idx.min(axis=0).tolist(), idx.max(axis=0).tolist())
    assert not bad, f"component: (max|diff|, points, index lo, index hi): {bad}"


def test_tb_active_and_bitwise_vs_oracle():
    p = sc_tb(ProductSim, profile=True)
    f = p._fields()
    info = f.tb_info()
    assert f.fused_active() and info["active"], info
    assert info["tb_items"] > 0 and info["rim_items"] > 0
    assert f.kernel_stats(5)[0] >= 4  # the two-step kernel ran (one launch per pair)
    _same(p, sc_tb(make_oracle))


@pytest.fixture(scope="module")
def oracle_tb():
    return sc_tb(make_oracle)


@pytest.mark.parametrize("schedule", [(("rim_zchunk", 12),), (("res", 16),), (("res_rim", 40),),
                                      (("res_tb2", 24), ("narrow", 0)), (("tb_ox", 60),),
                                      (("tb_ox", 60), ("tb_zchunk", 5)), (("tb_ox", 37),),
                                      (("tb_ox", 9), ("tb_zchunk", 3)), (("tb_px", 1),),
                                      (("tb_px", 1), ("tb_ox", 60))],
                         ids=["rim_zchunk12", "res16", "res_rim40", "res_tb2_24_wide", "ox60",
                              "ox60_z5", "ox37_odd_starts", "ox9_z3", "px1", "px1_ox60"])
def test_tb_schedule_options_bitwise(oracle_tb, schedule):
    """The scheduling options of Fields.set_schedule (rim item length, CUs left free by the
    pair launches, the strip body, two-step item widths -- 37 columns puts every other item's
    first column on an odd x (lane 0 three columns left of it, own ranges that start and end
    inside a lane's column pair: the 8-byte store paths), 9 columns many ragged items -- short
    two-step chunks, the round-5 one-column-per-lane kernel) change only how the same per-point
    arithmetic is laid out: bitwise the oracle."""
    p = sc_tb(ProductSim, profile=True, schedule=schedule)
    assert p._fields().tb_info()["active"] and p._fields().kernel_stats(5)[0] >= 4
    _same(p, oracle_tb)


def test_tb_interior_items_beside_previous_rim():
    """Narrow, short two-step items (9 columns, 3 planes): many have a footprint that meets no
    rim box, and one rank runs those on a third stream from the previous pair's middle guard on,
    beside its second rim launch (tb_lint).  Long batches of pairs, odd calls and a one-step
    step between them: bitwise the oracle and the same run with the option off."""
    sched = (("tb_ox", 9), ("tb_zchunk", 3))
    steps = (1, 24, 3, 1, 10)
    p = sc_tb(ProductSim, profile=True, schedule=sched + (("tb_lint", 1),), steps=steps)
    info = p._fields().tb_info()
    assert info["active"] and 0 < info["tb_interior_items"] < info["tb_items"], info
    _same(p, sc_tb(make_oracle, steps=steps))
    _same(p, sc_tb(ProductSim, schedule=sched, steps=steps))


def sc_tb_volume(make, big, steps=(1, 10, 1, 6), schedule=()):
    """sc_tb's slab with Ez volume currents inside L2: a 3.0 x 3.0 x 1.2 box (more D source points
    than one workgroup of the pair's source + guard launch takes: the two-launch fallback) or a
    plane given twice plus a point on it (several source layers in the one launch)."""
    o = vol(make, 3, [9.6, 6.4, 8.0], 10, center_origin=True)
    o.add_pml(0.7)
    for c in E_COMPS:
        x, y, z = o.coords(c)
        o.set_chi1inv(c, c, np.where((np.abs(y) < 0.8) & (z > -0.4) & (z < 3.0), 1.0 / 6.0, 1.0))
    if big:
        o.add_gaussian_volume_source(2, 0.25, 4.0, 0.0, 40.0, (-1.53, -1.47, -0.61), (1.51, 1.52, 0.63),
                                     0.5)  # > 30 x 30 x 12 points
    else:
        for a in (0.6, 0.2):
            o.add_gaussian_volume_source(2, 0.25, 4.0, 0.0, 40.0, (-1.0, -1.0, 0.33), (1.0, 1.0, 0.33), a)
        o.add_gaussian_source(2, 0.25, 4.0, 0.0, 40.0, (0.05, 0.05, 0.33), 1.0)
    random_init(o, (6, 7, 8, 9, 10, 11))
    if isinstance(o, ProductSim):
        for opt, val in schedule:
            o._fields().set_schedule(opt, val)
    for n in steps:
        o.step(n)
    return o


@pytest.mark.parametrize("big", [False, True], ids=["layers", "long_list"])
def test_tb_volume_sources_src_guard(big):
    """A pair's step sources and NaN guard in one launch (src_guard_kernel): several source
    layers in that launch, and the two-launch fallback for a long source list -- bitwise the
    oracle and the two-launch path."""
    p = sc_tb_volume(ProductSim, big)
    assert p._fields().tb_info()["active"]
    _same(p, sc_tb_volume(make_oracle, big))
    _same(p, sc_tb_volume(ProductSim, big, schedule=(("src_guard", 0),)))


def test_tb_equals_one_step_path():
    """Odd calls, one-step calls between pairs: identical to stepping one step at a time."""
    steps = (1, 7, 1, 4, 2, 3)
    _same(sc_tb(ProductSim, steps=steps), sc_tb(ProductSim, steps=steps, tb=False))


def test_tb_vacuum_no_chi1inv():
    kw = dict(eps=None, steps=(1, 9))
    _same(sc_tb(ProductSim, **kw), sc_tb(make_oracle, **kw))


def test_tb_f64_chi1inv():
    """More than 256 distinct chi1inv values: no palette, f64 chi1inv in the two-step kernel."""
    kw = dict(random_eps=True, steps=(1, 8))
    _same(sc_tb(ProductSim, **kw), sc_tb(make_oracle, **kw))


@pytest.mark.parametrize("zc", [1, 5, 200])
def test_tb_chunk_lengths(zc):
    """Two-step items of 1 plane (three halo planes per own plane), 5 and longer than L2."""
    os.environ["MNL_TB_ZCHUNK"] = str(zc)
    try:
        p = sc_tb(ProductSim, steps=(1, 6))
    finally:
        del os.environ["MNL_TB_ZCHUNK"]
    assert p._fields().tb_info()["active"]
    _same(p, sc_tb(make_oracle, steps=(1, 6)))


def test_tb_sources_on_hole_edges():
    """Source points on and next to L2's faces and corners, two in one hole, one in the
    x-alignment margin: the holes and the rim faces of the items around them."""
    srcs = ((-3.45, -1.75, -2.55), (-3.35, -1.65, -2.45), (3.05, 2.35, 2.95), (0.0, 0.0, 0.0),
            (0.05, 0.0, 0.0), (-3.85, 0.0, 0.0), (0.0, 2.55, 0.0))
    kw = dict(srcs=srcs, steps=(1, 11))
    _same(sc_tb(ProductSim, **kw), sc_tb(make_oracle, **kw))


def test_tb_no_source():
    kw = dict(srcs=(), steps=(1, 6))
    _same(sc_tb(ProductSim, **kw), sc_tb(make_oracle, **kw))


def test_tb_too_small_for_l2():
    """A grid whose lean box leaves no two-step region steps one step at a time."""
    p = sc_tb(ProductSim, sizes=(3.2, 3.2, 3.2), srcs=((0.05, 0.05, 0.05),), steps=(1, 4))
    assert not p._fields().tb_info()["active"]
    _same(p, sc_tb(make_oracle, sizes=(3.2, 3.2, 3.2), srcs=((0.05, 0.05, 0.05),), steps=(1, 4)))


def test_tb_long_batch():
    """Many pairs in one batch, an odd step at the end (one step), NaN guards inside."""
    kw = dict(steps=(1, 125))
    _same(sc_tb(ProductSim, **kw), sc_tb(make_oracle, **kw))


@pytest.mark.parametrize("sizes", [(9.6, 6.4, 8.0), (9.6, 16.0, 6.4)])
def test_tb_narrow_strips(sizes):
    """PML 1.0 (10 cells): L2 starts 16 columns from the low x face, so both x-face rim strips
    are 16 columns wide and run in the narrow strip body (the left one without an x-1 column,
    the right one reading the new B of its x-1 column from the two-step kernel's stores);
    16.0 in y gives three row blocks per strip.  Bitwise the oracle and the wide-strip path."""
    kw = dict(sizes=sizes, dpml=1.0, steps=(1, 10, 3), srcs=SRCS[:1] + SRCS[3:])
    p = sc_tb(ProductSim, profile=True, **kw)
    info = p._fields().tb_info()
    assert info["active"] and info["narrow_items"] >= 2, info
    _same(p, sc_tb(make_oracle, **kw))
    os.environ["MNL_TB_NARROW"] = "0"
    try:
        q = sc_tb(ProductSim, **kw)
    finally:
        del os.environ["MNL_TB_NARROW"]
    assert q._fields().tb_info()["narrow_items"] == 0
    _same(p, q)


@pytest.mark.parametrize("group", [GroupSim, GroupSim3])
def test_tb_slabs(group):
    """z-slabs of one grid (in-process transport): every rank steps pairs (L2 >= 2 planes
    from its slab faces, the faces in the rim: B/H and E plane exchanges of the middle and
    new sets, the top plane's shell kernels between them), bitwise the oracle."""
    kw = dict(sizes=(9.6, 6.4, 9.6), steps=(1, 12, 1, 3))
    p = sc_tb(group, **kw)
    assert all(f.tb_info()["active"] for f in p._all())
    _same(p, sc_tb(make_oracle, **kw))


def test_tb_slabs_equal_one_step():
    kw = dict(sizes=(9.6, 6.4, 9.6), steps=(1, 7, 2, 1, 6))
    _same(sc_tb(GroupSim3, **kw), sc_tb(GroupSim3, tb=False, **kw))


def test_tb_dft_flux():
    """DFT flux monitors with pairs of steps: the middle step is sampled from the mid set
    (the two-step items store step n+1 of the points the samples average), the second from
    the new state; every per-point DFT value bitwise the oracle's (src/dft.cpp:249-300)."""
    from scenarios import sc_flux_3d
    from test_gpu_dft import _same_dft
    kw = dict(sizes=[9.6, 6.4, 8.0], steps=24)
    p, hs = sc_flux_3d(ProductSim, **kw)
    assert p._fields().tb_info()["active"]  # the last call stepped pairs
    o, _ = sc_flux_3d(make_oracle, **kw)
    _same_dft(p, o, hs)


@pytest.mark.parametrize("group", [GroupSim, GroupSim3])
def test_tb_slabs_dft_flux(group):
    """z-slabs with DFT flux monitors (round 6: multi-rank runs with monitors step pairs too):
    the middle step is sampled once the slab-face chain has put mid's top plane, sources and
    E ghost in and mid's H component normal to the slabs has its low ghost (exchange kind 3);
    the flux monitors cross the slab faces.  Per-point DFT values bitwise the oracle, the flux
    sums within 1e-12 (sum over ranks), the fields bitwise."""
    from scenarios import sc_flux_3d
    from test_gpu_dft import _same_dft
    kw = dict(sizes=[9.6, 6.4, 9.6], steps=24)
    p, hs = sc_flux_3d(group, **kw)
    assert all(f.tb_info()["active"] for f in p._all())
    o, _ = sc_flux_3d(make_oracle, **kw)
    _same_dft(p, o, hs, flux_exact=False)
    _same(p, o)


def test_tb_dft_compact_fallbacks(monkeypatch):
    """The pairs' samples of two-step points come from the monitors' compact boxes (DESIGN.md
    section 10); the paths around them stay bitwise the oracle: compact boxes switched off
    (MNL_DFT_CMP=0: the middle state in the mid set), and a fifth monitor beyond the four
    compact boxes, added half-way (its middle state in the mid set, the others compact)."""
    from scenarios import FLUX3D_FREQS, sc_flux_3d
    from test_gpu_dft import _same_dft
    kw = dict(sizes=[9.6, 6.4, 8.0], steps=24)
    o, hs = sc_flux_3d(make_oracle, **kw)
    monkeypatch.setenv("MNL_DFT_CMP", "0")
    p, _ = sc_flux_3d(ProductSim, **kw)
    monkeypatch.delenv("MNL_DFT_CMP")
    assert p._fields().tb_info()["active"]
    _same_dft(p, o, hs)

    def fifth(sim):
        hy, hz = 0.5 * kw["sizes"][1], 0.5 * kw["sizes"][2]
        sim.add_dft_flux([([-0.9, -hy, -hz], [-0.9, hy, hz], 0, 1.0)], FLUX3D_FREQS, 1)

    o5, hs5 = sc_flux_3d(make_oracle, extra=fifth, **kw)
    p5, _ = sc_flux_3d(ProductSim, extra=fifth, **kw)
    assert p5._fields().tb_info()["active"]
    _same_dft(p5, o5, hs5 + [len(hs5)])


def test_tb_dft_fields():
    """DFT field monitors (whole-cell components, boxes across PML chunks, planes, lines)
    with pairs of steps: bitwise the oracle."""
    from scenarios import sc_dft_fields_3d
    from test_gpu_dft_fields import _same as same_fields
    kw = dict(sizes=[9.6, 6.4, 8.0], steps=20)
    p, objs = sc_dft_fields_3d(ProductSim, **kw)
    assert p._fields().tb_info()["active"]  # the last call stepped pairs
    o, _ = sc_dft_fields_3d(make_oracle, **kw)
    same_fields(p, o, objs)


def test_tb_middle_set_oom_fallback():
    """When the middle buffer set does not fit (MNL_TB_OOM=1 simulates the failed hipMalloc),
    temporal blocking switches itself off and the fields step one step at a time, bitwise
    the oracle, instead of failing the step."""
    os.environ["MNL_TB_OOM"] = "1"
    try:
        p = sc_tb(ProductSim, steps=(1, 9, 4))
    finally:
        del os.environ["MNL_TB_OOM"]
    info = p._fields().tb_info()
    assert not info["active"] and not info["enabled"], info
    _same(p, sc_tb(make_oracle, steps=(1, 9, 4)))
