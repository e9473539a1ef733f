"""Oracle array slices (fields::get_array_slice, src/array_slice.cpp:251-704,
loop_in_chunks weights src/loop_in_chunks.cpp:257-300): the reference holds no
golden slice for real fields without MPB/HDF5 (python/tests/test_get_array*.py
need eigenmode sources or h5 files), so the restatement is checked against its
defining properties: Centered-grid averages, shapes, linear interpolation of
empty dimensions, and chunk-boundary independence."""
import numpy as np

from scenarios import make_oracle, sc_cfg1, sc_vacuum_pml_3d


def test_whole_cell_is_centered_average():
    o = sc_cfg1(make_oracle, steps=120)
    a = o.get_array_slice(2, [-10, -10, 0], [10, 10, 0])
    assert a.shape == (200, 200)
    ez = o.get_array(2)  # Yee layout (201 x 201), Ez unshifted in x and y
    ref = 0.25 * (ez[:-1, :-1] + ez[1:, :-1] + ez[:-1, 1:] + ez[1:, 1:])
    np.testing.assert_allclose(a, ref, rtol=1e-13, atol=1e-300)


def test_empty_dimension_interpolates_linearly():
    o = sc_cfg1(make_oracle, steps=120)
    # centered points at y = (k + 0.5)/10; y = 0.33 lies between 0.25 and 0.35
    a = o.get_array_slice(2, [-10, 0.25, 0], [10, 0.25, 0])
    b = o.get_array_slice(2, [-10, 0.35, 0], [10, 0.35, 0])
    m = o.get_array_slice(2, [-10, 0.33, 0], [10, 0.33, 0])
    assert m.shape == (200,)
    np.testing.assert_allclose(m, 0.2 * a + 0.8 * b, rtol=1e-9, atol=1e-18)


def test_3d_slices_shapes_and_chunks():
    """A plane and a box crossing PML chunk boundaries: the values on either side
    of a chunk boundary come from different chunks but form one array."""
    o = sc_vacuum_pml_3d(make_oracle, steps=40)
    pl = o.get_array_slice(0, [-1.6, -1.6, 0.12], [1.6, 1.6, 0.12])
    assert pl.shape == (32, 32)
    box = o.get_array_slice(1, [-1.2, -0.65, -1.0], [0.9, 0.45, 0.3])
    assert box.ndim == 3 and np.isfinite(box).all() and np.abs(box).max() > 0
    pt = o.get_array_slice(2, [0.05, 0.05, 0.05], [0.05, 0.05, 0.05])
    assert np.ndim(pt) == 0


def test_snap_picks_nearest_plane():
    """snap_empty_dimensions (loop_in_chunks.cpp:275-287): y = 0.33 snaps to the
    centered plane y = 0.35 (the nearer one), unweighted."""
    o = sc_cfg1(make_oracle, steps=120)
    b = o.get_array_slice(2, [-10, 0.35, 0], [10, 0.35, 0])
    s = o.get_array_slice(2, [-10, 0.33, 0], [10, 0.33, 0], snap=True)
    assert s.shape == (200,)
    np.testing.assert_array_equal(s, b)
