"""Low-level mirror of the reference C++ API (meep::structure / meep::fields).

Mirrors src/meep.hpp:809-920 (structure) and 1731-2330 (fields) for the
hot-path subset: grid_volume construction (vol1d/vol2d/vol3d +
center_origin), pml(), set_chi1inv / set_epsilon, set_chi2 / set_chi3,
add_susceptibility(lorentzian), add_point_source / add_volume_source (point),
step(), time()/round_time(), get_field(), and raw component arrays.

Arrays use the reference's own per-chunk layout for the whole cell
((n+1) points per present direction, Z fastest; src/vec.cpp:482-494).
"""
import ctypes
import os
import math

import numpy as np

from . import _lib
from ._lib import check, dptr, lib, ptr

Ex, Ey, Ez, Hx, Hy, Hz, Dx, Dy, Dz, Bx, By, Bz = range(12)
Dielectric, Permeability = 12, 13  # derived slice components (src/meep/vec.hpp:52-53)
X, Y, Z = 0, 1, 2

# meep::time_sink (src/meep.hpp:1610-1633) and the print_times labels
# (DescriptionByTimeSink, src/time.cpp:28-51), in enum order
TIME_SINKS = (
    ("Connecting", "connecting chunks"), ("Stepping", "time stepping"),
    ("Boundaries", "copying boundaries"), ("MpiAllTime", "all-all communication"),
    ("MpiOneTime", "1-1 communication"), ("FieldOutput", "outputting fields"),
    ("FourierTransforming", "Fourier transforming"), ("MPBTime", "MPB mode solver"),
    ("GetFarfieldsTime", "far-field transform"), ("Other", "everything else"),
    ("FieldUpdateB", "updating B field"), ("FieldUpdateH", "updating H field"),
    ("FieldUpdateD", "updating D field"), ("FieldUpdateE", "updating E field"),
    ("BoundarySteppingB", "boundary stepping B"), ("BoundarySteppingWH", "boundary stepping WH"),
    ("BoundarySteppingPH", "boundary stepping PH"), ("BoundarySteppingH", "boundary stepping H"),
    ("BoundarySteppingD", "boundary stepping D"), ("BoundarySteppingWE", "boundary stepping WE"),
    ("BoundarySteppingPE", "boundary stepping PE"), ("BoundarySteppingE", "boundary stepping E"),
)


def set_verbosity(level):
    """meep::verbosity of the native library (rank 0's "on time step" lines)."""
    lib().mnl_set_verbosity(int(level))


def get_verbosity():
    return lib().mnl_get_verbosity()
COMPONENT_NAMES = ["ex", "ey", "ez", "hx", "hy", "hz", "dx", "dy", "dz", "bx", "by", "bz"]


class GridVolume:
    """grid_volume for Cartesian D1 (Z), D2 (X,Y), D3 (X,Y,Z)."""

    def __init__(self, dim, n, a, io=(0, 0, 0)):
        self.dim = int(dim)
        self.has = [dim >= 2, dim >= 2, dim != 2]
        self.n = [int(n[d]) if self.has[d] else 0 for d in range(3)]
        self.io = [int(io[d]) if self.has[d] else 0 for d in range(3)]
        self.a = float(a)

    @classmethod
    def vol(cls, dim, sizes, a, center_origin=False):
        """vol1d/vol2d/vol3d (src/vec.cpp:904-931) [+ center_origin (vec.hpp:1150)]."""
        n = [0, 0, 0]
        if dim == 1:
            n[2] = int(sizes[0] * a + 0.5)
        elif dim == 2:
            n[0] = 1 if sizes[0] == 0 else int(sizes[0] * a + 0.5)
            n[1] = 1 if sizes[1] == 0 else int(sizes[1] * a + 0.5)
        else:
            n = [1 if s == 0 else int(s * a + 0.5) for s in sizes]
        io = [-(v - (v & 1)) for v in n] if center_origin else [0, 0, 0]
        return cls(dim, n, a, io)

    def shape(self):
        return tuple(self.n[d] + 1 for d in range(3) if self.has[d])

    def ntot(self):
        return int(np.prod(self.shape()))

    def shift(self, c, d):
        if not self.has[d]:
            return 0
        t = c // 3
        if t in (0, 2):
            return 1 if d == c % 3 else 0
        return 1 if d != c % 3 else 0

    def coords(self, c):
        axes = []
        for d in range(3):
            if self.has[d]:
                j = np.arange(self.n[d] + 1)
                axes.append((self.io[d] + 2 * j + self.shift(c, d)) * (0.5 / self.a))
        return np.meshgrid(*axes, indexing="ij")

    def center(self):
        """grid_volume::center() (src/vec.cpp:1089-1103)."""
        out = []
        for d in range(3):
            if self.has[d]:
                n = self.n[d] - (self.n[d] & 1)
                out.append((self.io[d] + n) * (0.5 / self.a))
            else:
                out.append(0.0)
        return out


class Structure:
    """meep::structure for one grid_volume (no symmetry, PML chunks implicit)."""

    def __init__(self, gv, courant=0.5):
        self.gv = gv
        self.courant = float(courant)
        na = (ctypes.c_int * 3)(*gv.n)
        ia = (ctypes.c_int * 3)(*gv.io)
        self.h = lib().mnl_structure_create(gv.dim, na, gv.a, self.courant, ia)
        if not self.h:
            raise RuntimeError(lib().mnl_last_error().decode())
        self._nsus = 0

    def __del__(self):
        if getattr(self, "h", None):
            lib().mnl_structure_destroy(self.h)
            self.h = None

    def add_pml(self, thickness, dirs=(0, 1, 2), sides=(0, 1), R=1e-15, mean_stretch=1.0):
        for d in dirs:
            for s in sides:
                check(lib().mnl_structure_add_pml(self.h, d, s, float(thickness), R, mean_stretch))

    def _arr(self, a):
        return np.ascontiguousarray(np.broadcast_to(a, self.gv.shape()), dtype=np.float64).ravel()

    def set_chi1inv(self, comp, d, arr):
        check(lib().mnl_structure_set_chi1inv(self.h, comp, d, None if arr is None else ptr(self._arr(arr))))

    def set_epsilon_fn(self, fn):
        """set_epsilon without averaging: chi1inv = 1/eps(location) per E component."""
        for c in (Ex, Ey, Ez):
            if self.gv.dim == 1 and c != Ex:
                continue
            self.set_chi1inv(c, c % 3, 1.0 / fn(*self.gv.coords(c)))

    def set_mu_fn(self, fn):
        """structure::set_mu without averaging: chi1inv of the H components =
        1/mu(location) (set_chi1inv(H_stuff), src/anisotropic_averaging.cpp:221-298)."""
        for c in (Hx, Hy, Hz):
            if self.gv.dim == 1 and c != Hy:
                continue
            self.set_chi1inv(c, c % 3, 1.0 / fn(*self.gv.coords(c)))

    def set_epsilon_geometry(self, objects, default_eps=1.0, use_anisotropic_averaging=True,
                             tol=1e-4, maxeval=100000, device=-1):
        """structure::set_epsilon(material_function &, use_anisotropic_averaging, tol,
        maxeval) (src/structure.cpp:397-401; subpixel averaging of
        src/anisotropic_averaging.cpp:58-298) for a material function made of
        geometric objects, computed on a HIP device.  objects: rows
        {kind, eps, cx, cy, cz, p0, p1, p2} (include/meep_nl_amd.h), later rows win."""
        o = np.ascontiguousarray(np.asarray(objects, dtype=np.float64).reshape(-1, 8))
        check(lib().mnl_structure_set_epsilon_geometry(
            self.h, int(device), o.shape[0], ptr(o) if o.shape[0] else None, float(default_eps),
            int(bool(use_anisotropic_averaging)), float(tol), int(maxeval)))

    def get_chi1inv(self, comp, d):
        """chi1inv[comp][d] over the whole cell (canonical layout); None if trivial."""
        out = np.empty(self.gv.shape(), dtype=np.float64)
        rc = lib().mnl_structure_get_chi1inv(self.h, comp, d, ptr(out))
        if rc == 1:
            return None
        check(rc)
        return out

    def set_chi2(self, comp, arr):
        check(lib().mnl_structure_set_chi2(self.h, comp, ptr(self._arr(arr))))

    def set_chi3(self, comp, arr):
        check(lib().mnl_structure_set_chi3(self.h, comp, ptr(self._arr(arr))))

    def set_conductivity(self, comp, arr):
        """structure::set_conductivity(c, C) (src/structure.cpp:868-905): D or B
        component (E / H name their D / B array; E values are multiplied by the
        diagonal chi1inv set so far).  None resets to zero."""
        a = None if arr is None else self._arr(arr)
        check(lib().mnl_structure_set_conductivity(self.h, comp, None if a is None else ptr(a)))

    def dump(self, fname):
        """structure::dump (src/structure_dump.cpp): the host-side material
        description (flat binary, not HDF5)."""
        check(lib().mnl_structure_dump(self.h, os.fsencode(fname)))

    def load(self, fname):
        """structure::load: replace the materials / PML / susceptibilities by a
        dumped description of the same grid volume (before creating fields)."""
        check(lib().mnl_structure_load(self.h, os.fsencode(fname)))

    def add_lorentzian(self, omega0, gamma, sigmas, drude=False):
        s = [None if v is None else self._arr(v) for v in sigmas]
        check(lib().mnl_structure_add_lorentzian(self.h, omega0, gamma, int(drude),
                                                 *[ptr(v) for v in s]))
        self._nsus += 1
        return self._nsus - 1

    def add_lorentzian_tensor(self, omega0, gamma, sigma, drude=False):
        """add_susceptibility with a sigma tensor (src/anisotropic_averaging.cpp:
        300-372): sigma[c][d] (3x3 nested, None = 0) per E component row c at c's
        Yee points; off-diagonal entries sampled half a pixel back along c."""
        arrs = [None if sigma[c][d] is None else self._arr(sigma[c][d])
                for c in range(3) for d in range(3)]
        ptrs = (dptr * 9)(*[ptr(a) if a is not None else None for a in arrs])
        check(lib().mnl_structure_add_lorentzian_tensor(self.h, float(omega0), float(gamma),
                                                         int(drude), ptrs))

    def add_magnetic_lorentzian(self, omega0, gamma, sigmas, drude=False):
        """add_susceptibility(sigma, H_stuff, lorentzian_susceptibility): diagonal
        sigma per H component at its Yee points (None = 0)."""
        s = [None if v is None else self._arr(v) for v in sigmas]
        check(lib().mnl_structure_add_magnetic_lorentzian(self.h, float(omega0), float(gamma),
                                                          int(drude), *[ptr(v) for v in s]))

    def set_box(self, kind, box, value, index=0):
        b = np.ascontiguousarray(box, dtype=np.float64)
        check(lib().mnl_structure_set_box(self.h, kind, index, ptr(b), float(value)))

    def set_nonlinear_mode(self, mode):
        """'fork' (default: chi2 through Newton-Raphson, chi3 inert) or 'upstream'
        (upstream Meep's Pade chi2/chi3 update, src/step_generic.cpp:546-553)."""
        m = {"fork": 0, "upstream": 1}[mode] if isinstance(mode, str) else int(mode)
        check(lib().mnl_structure_set_nonlinear_mode(self.h, m))


def _src_last_time(kind, params):
    """src_time::last_time(): gaussian float(peak_time + cutoff) with the cutoff
    shrink of gaussian_src_time(f, w, st, et) (src/sources.cpp:85-96,
    src/meep.hpp:1024); continuous end_time (src/meep.hpp:1046)."""
    if kind == 0:
        w, st, et = params[1], params[2], params[3]
        peak, cutoff = 0.5 * (st + et), (et - st) * 0.5
        while math.exp(-cutoff * cutoff / (2 * w * w)) < 1e-100:
            cutoff *= 0.9
        cutoff = float(np.float32(cutoff))
        return float(np.float32(peak + cutoff))
    return float(params[4])


class Fields:
    """meep::fields with use_real_fields() on one MI355X (or one z-slab of it)."""

    def __init__(self, structure, device=-1, rank=0, nranks=1, nccl_id=None, hub=None):
        self.s = structure
        self.gv = structure.gv
        if nranks > 1 and hub is not None:
            self.h = lib().mnl_fields_create_local(structure.h, device, rank, nranks, hub.h)
        elif nranks > 1:
            self.h = lib().mnl_fields_create_dist(structure.h, device, rank, nranks, nccl_id)
        else:
            self.h = lib().mnl_fields_create(structure.h, device)
        if not self.h:
            raise RuntimeError(lib().mnl_last_error().decode())
        self.rank, self.nranks = rank, nranks
        self._hub = hub  # the hub must outlive the fields of its slabs

    def __del__(self):
        if getattr(self, "h", None):
            lib().mnl_fields_destroy(self.h)
            self.h = None

    # -- sources
    def add_point_source(self, comp, kind, params, pos, amp=1.0, is_integrated=False):
        p = np.ascontiguousarray(params, dtype=np.float64)
        pos = np.ascontiguousarray(list(pos) + [0.0] * (3 - len(pos)), dtype=np.float64)
        amp = complex(amp)
        check(lib().mnl_fields_add_point_source(self.h, comp, kind, ptr(p), len(p), ptr(pos),
                                                amp.real, amp.imag, int(is_integrated)))
        self._last_times = getattr(self, "_last_times", [])
        self._last_times.append(_src_last_time(kind, list(params)))

    def add_custom_source(self, comp, func, start, end, pos, amp=1.0, is_integrated=False):
        """custom_src_time(func, data, start, end) (src/meep.hpp:1059-1092): func(t) ->
        complex dipole, called on the host at every step.  One callback per Python
        function, so sources sharing a function merge as in custom_src_time::is_equal."""
        cbs = self.__dict__.setdefault("_custom_cbs", {})
        if id(func) not in cbs:
            def _cb(t, _data, re, im, func=func):
                v = complex(func(t))
                re[0] = v.real
                im[0] = v.imag
            cbs[id(func)] = (func, _lib.SRC_FUNC(_cb))
        cf = cbs[id(func)][1]
        pos = np.ascontiguousarray(list(pos) + [0.0] * (3 - len(pos)), dtype=np.float64)
        amp = complex(amp)
        check(lib().mnl_fields_add_custom_point_source(self.h, comp, cf, None, float(start),
                                                       float(end), ptr(pos), amp.real, amp.imag,
                                                       int(is_integrated)))
        self._last_times = getattr(self, "_last_times", [])
        self._last_times.append(float(np.float32(end)))

    def _amp_cb(self, amp_func):
        """ctypes callback for a volume source's amplitude function A(r) (r relative
        to the volume centre, 3 coordinates) -> complex; kept alive with the fields."""
        if amp_func is None:
            return _lib.AMP_FUNC()
        def _cb(rel, _data, re, im, f=amp_func):
            v = complex(f((rel[0], rel[1], rel[2])))
            re[0] = v.real
            im[0] = v.imag
        cb = _lib.AMP_FUNC(_cb)
        self.__dict__.setdefault("_amp_cbs", []).append(cb)
        return cb

    def add_volume_source(self, comp, kind, params, vmin, vmax, amp=1.0, is_integrated=False,
                          amp_func=None):
        """fields::add_volume_source(c, src, volume(vmin, vmax), A, amp)
        (src/sources.cpp:455-494); amp_func(r) -> complex, r relative to the centre."""
        p = np.ascontiguousarray(params, dtype=np.float64)
        lo = np.ascontiguousarray(list(vmin) + [0.0] * (3 - len(vmin)), dtype=np.float64)
        hi = np.ascontiguousarray(list(vmax) + [0.0] * (3 - len(vmax)), dtype=np.float64)
        amp = complex(amp)
        check(lib().mnl_fields_add_volume_source(self.h, comp, kind, ptr(p), len(p), ptr(lo),
                                                 ptr(hi), amp.real, amp.imag, int(is_integrated),
                                                 self._amp_cb(amp_func), None))
        self._last_times = getattr(self, "_last_times", [])
        self._last_times.append(_src_last_time(kind, list(params)))

    def add_custom_volume_source(self, comp, func, start, end, vmin, vmax, amp=1.0,
                                 is_integrated=False, amp_func=None):
        cbs = self.__dict__.setdefault("_custom_cbs", {})
        if id(func) not in cbs:
            def _cb(t, _data, re, im, func=func):
                v = complex(func(t))
                re[0] = v.real
                im[0] = v.imag
            cbs[id(func)] = (func, _lib.SRC_FUNC(_cb))
        lo = np.ascontiguousarray(list(vmin) + [0.0] * (3 - len(vmin)), dtype=np.float64)
        hi = np.ascontiguousarray(list(vmax) + [0.0] * (3 - len(vmax)), dtype=np.float64)
        amp = complex(amp)
        check(lib().mnl_fields_add_custom_volume_source(
            self.h, comp, cbs[id(func)][1], None, float(start), float(end), ptr(lo), ptr(hi),
            amp.real, amp.imag, int(is_integrated), self._amp_cb(amp_func), None))
        self._last_times = getattr(self, "_last_times", [])
        self._last_times.append(float(np.float32(end)))

    def add_gaussian_volume_source(self, comp, freq, width, start, end, vmin, vmax, amp=1.0,
                                   is_integrated=False, amp_func=None):
        self.add_volume_source(comp, 0, [freq, width, start, end], vmin, vmax, amp, is_integrated,
                               amp_func)

    def add_gaussian_source(self, comp, freq, width, start, end, pos, amp=1.0,
                            is_integrated=False):
        """gaussian_src_time(f, w, start, end) (src/sources.cpp:85-96)."""
        self.add_point_source(comp, 0, [freq, width, start, end], pos, amp, is_integrated)

    def add_continuous_source(self, comp, freq, width, start, end, slowness, pos, amp=1.0,
                              is_integrated=False):
        f = complex(freq)
        self.add_point_source(comp, 1, [f.real, f.imag, width, start, end, slowness], pos, amp,
                              is_integrated)

    def legacy_point_source(self, comp, freq, width, peaktime, cutoff, pos, amp):
        """Deprecated C++ fields::add_point_source(c, freq, width, peaktime, cutoff,
        vec, amp) (src/sources.cpp:189-211); C++ sources are integrated by default
        (src/meep.hpp:950-951), magnetic ones are not."""
        width = width / freq
        dt = self.dt
        cutoff = (1.0 / self.gv.a) + cutoff * width
        if peaktime <= 0.0:
            peaktime = self.t * dt + cutoff
        peaktime += (-dt * 0.5) if comp in (Hx, Hy, Hz) else dt
        self.add_gaussian_source(comp, freq, width, peaktime - cutoff, peaktime + cutoff, pos,
                                 amp, is_integrated=comp not in (Hx, Hy, Hz))

    def require_component(self, comp):
        check(lib().mnl_fields_require_component(self.h, comp))

    def initialize_field(self, comp, values):
        """fields::initialize_field(c, func) (src/initialize.cpp:135-161): values is
        the whole-cell array of func at the points of comp (real part used), or a
        callable f(*coords) vectorised over the coordinate arrays of comp."""
        if callable(values):
            values = values(*self.gv.coords(comp))
        v = np.ascontiguousarray(np.real(np.broadcast_to(values, self.gv.shape())),
                                 dtype=np.float64).ravel()
        check(lib().mnl_fields_initialize_field(self.h, comp, ptr(v), v.size))

    def set_nan_check(self, every):
        """NaN / Inf guard cadence in steps (src/step.cpp:138-139 checks every step)."""
        check(lib().mnl_fields_set_nan_check(self.h, int(every)))

    def last_source_time(self):
        """fields::last_source_time (src/bands.cpp:35-41): latest src_time::last_time()."""
        return max([0.0] + getattr(self, "_last_times", []))

    # -- stepping
    def step(self, n=1):
        check(lib().mnl_fields_step(self.h, int(n)))

    def tune(self, reps=8):
        """Time the fused step's knobs over real steps and keep the fastest (mnl_fields_tune:
        the tile kernel's z-chunk length, then on one rank with polarization chunks the CUs
        of their general kernel beside the tile kernel; with temporal blocking the planes and
        widths of its two-step items).  Every candidate runs two warm-up steps and reps
        (rounded up to even) timed ones: at most 2 + 32 * (2 + reps) steps, results identical
        to plain stepping (round 6: 8 timed steps by default, 4 gave choices off by up to 10 %
        at 256^3).  Returns (zchunk, gen_cus); -1 = not tuned (not in the fused tile mode)."""
        z, g = ctypes.c_int(0), ctypes.c_int(0)
        check(lib().mnl_fields_tune(self.h, int(reps), ctypes.byref(z), ctypes.byref(g)))
        return z.value, g.value

    def _time(self):
        t = ctypes.c_longlong()
        dt = ctypes.c_double()
        check(lib().mnl_fields_time(self.h, ctypes.byref(t), ctypes.byref(dt)))
        return t.value, dt.value

    @property
    def t(self):
        return self._time()[0]

    @t.setter
    def t(self, value):  # the SWIG binding's fields.t assignment
        check(lib().mnl_fields_set_time(self.h, int(value)))

    def zero_fields(self):
        """fields::zero_fields (src/fields.cpp:638-664); DFT accumulators are kept."""
        check(lib().mnl_fields_zero_fields(self.h))

    def remove_sources(self):
        """fields::remove_sources (src/fields.cpp:601-610)."""
        check(lib().mnl_fields_remove_sources(self.h))
        self._last_times = []

    @property
    def dt(self):
        return self._time()[1]

    def time(self):
        t, dt = self._time()
        return t * dt

    def round_time(self):
        t, dt = self._time()
        return float(np.float32(t * dt))

    # -- energy (src/energy_and_flux.cpp:48-178)
    def _energy(self, which, vmin=None, vmax=None):
        out = ctypes.c_double()
        lo = None if vmin is None else np.ascontiguousarray(vmin, dtype=np.float64)
        hi = None if vmax is None else np.ascontiguousarray(vmax, dtype=np.float64)
        check(lib().mnl_fields_energy_in_box(self.h, which, ptr(lo), ptr(hi), ctypes.byref(out)))
        return out.value

    def electric_energy_in_box(self, vmin=None, vmax=None):
        """fields::electric_energy_in_box: sum over E comps of (1/2) integral E.D."""
        return self._energy(0, vmin, vmax)

    def magnetic_energy_in_box(self, vmin=None, vmax=None):
        """fields::magnetic_energy_in_box with the current (unsynchronized) B, H."""
        return self._energy(1, vmin, vmax)

    def field_energy_in_box(self, vmin=None, vmax=None):
        """fields::field_energy_in_box: electric + magnetic energy of B / H
        synchronized to E's time (synchronize_magnetic_fields)."""
        return self._energy(2, vmin, vmax)

    def field_energy(self):
        """fields::field_energy (src/energy_and_flux.cpp:48): the whole cell."""
        return self._energy(2)

    # -- monitors
    def get_field(self, comp, pos):
        pos = np.ascontiguousarray(list(pos) + [0.0] * (3 - len(pos)), dtype=np.float64)
        out = ctypes.c_double()
        check(lib().mnl_fields_get_field(self.h, comp, ptr(pos), ctypes.byref(out)))
        return out.value

    def get_array(self, comp):
        nt = lib().mnl_fields_ntot(self.h)
        out = np.zeros(nt, dtype=np.float64)
        check(lib().mnl_fields_copy_component(self.h, comp, ptr(out), nt))
        return out.reshape(self.gv.shape())

    def get_array_slice(self, comp, vmin, vmax, snap=False):
        """fields::get_array_slice(volume, c) (src/array_slice.cpp:611-704) over
        [vmin, vmax] (3 coordinates): Centered-grid values, empty dimensions
        interpolated and collapsed; shape = kept directions in X, Y, Z order."""
        lo = np.ascontiguousarray(vmin, dtype=np.float64)
        hi = np.ascontiguousarray(vmax, dtype=np.float64)
        rank = ctypes.c_int(0)
        dims = (ctypes.c_longlong * 3)()
        check(lib().mnl_fields_array_slice(self.h, comp, ptr(lo), ptr(hi), int(snap),
                                           ctypes.byref(rank), dims, None, 0))
        shape = tuple(dims[k] for k in range(rank.value))
        out = np.zeros(int(np.prod(shape)) if shape else 1)
        check(lib().mnl_fields_array_slice(self.h, comp, ptr(lo), ptr(hi), int(snap),
                                           ctypes.byref(rank), dims, ptr(out), out.size))
        return out.reshape(shape) if shape else out[0]

    def center(self):
        return self.gv.center()

    # -- instrumentation
    def timers(self):
        out = np.zeros(6)
        check(lib().mnl_fields_timers(self.h, ptr(out)))
        return dict(zip(["FieldUpdateB", "FieldUpdateH", "FieldUpdateD", "FieldUpdateE",
                         "Sources", "BoundarySteppingHalo"], out.tolist()))

    def time_spent(self):
        """This rank's seconds per time sink, in meep::time_sink order
        (TIME_SINKS; mnl_fields_time_spent)."""
        out = np.zeros(len(TIME_SINKS))
        check(lib().mnl_fields_time_spent(self.h, ptr(out)))
        return out

    def reset_timers(self):
        check(lib().mnl_fields_reset_timers(self.h))

    def sum_to_all(self, values):
        """Sum of a float64 vector over the ranks of distributed fields (collective)."""
        v = np.ascontiguousarray(values, dtype=np.float64).copy()
        check(lib().mnl_fields_allreduce(self.h, ptr(v), v.size))
        return v

    def nr_fallbacks(self):
        v = ctypes.c_longlong()
        check(lib().mnl_fields_nr_fallbacks(self.h, ctypes.byref(v)))
        return v.value

    def transport(self):
        """'single', 'rccl', 'ipc' or 'local' (how ghost planes travel)."""
        return lib().mnl_fields_transport(self.h).decode()

    def fused_active(self):
        v = ctypes.c_int()
        check(lib().mnl_fields_mode(self.h, ctypes.byref(v)))
        return bool(v.value & 1)

    def tile_mode(self):
        """True if the fused step runs as one tile kernel (lean + PML bodies)."""
        v = ctypes.c_int()
        check(lib().mnl_fields_mode(self.h, ctypes.byref(v)))
        return bool(v.value & 16)

    def fused_concurrent(self):
        """True if the last fused step ran the polarization chunks' general kernel beside the
        tile (or lean) kernel on a CU split: kernel_stats(0) then spans both launches."""
        v = ctypes.c_int()
        check(lib().mnl_fields_mode(self.h, ctypes.byref(v)))
        return bool(v.value & 32)

    def fused_palette(self):
        """True if the fused kernel reads chi1inv through the byte palette."""
        v = ctypes.c_int()
        check(lib().mnl_fields_mode(self.h, ctypes.byref(v)))
        return bool(v.value & 2)

    def alloc_info(self):
        """(contiguous field allocations requested, requests that fell back)."""
        v = ctypes.c_int()
        check(lib().mnl_fields_mode(self.h, ctypes.byref(v)))
        return bool(v.value & 4), (v.value >> 8) & 255

    def set_fused(self, allow=True):
        check(lib().mnl_fields_set_fused(self.h, int(allow)))

    def set_profiling(self, on=True):
        check(lib().mnl_fields_set_profiling(self.h, int(on)))

    def kernel_stats(self, which=0):
        n = ctypes.c_longlong()
        ms = ctypes.c_double()
        b = ctypes.c_double()
        check(lib().mnl_fields_kernel_stats(self.h, which, ctypes.byref(n), ctypes.byref(ms),
                                            ctypes.byref(b)))
        return n.value, ms.value, b.value

    def set_temporal_blocking(self, on=True):
        """Allow / forbid stepping pairs of steps with the two-step kernel (identical
        results either way)."""
        check(lib().mnl_fields_set_temporal_blocking(self.h, 1 if on else 0))

    def set_schedule(self, which, value):
        """Scheduling option (identical results): 'narrow' = the narrow x-face strip body of
        the temporal-blocking rim, 'dft_pal' = DFT sampling plans carrying chi1inv as palette
        bytes, 'res' / 'res_tb2' / 'res_rim' = CUs left free by the pair launches (an integer;
        -1 the default), 'dft_cmp' = pairs sample DFT monitors from the two-step kernel's compact
        boxes, 'rim_zchunk' = planes per rim item of a pair (an integer; 0 the one-step chunk),
        'nr_early' = the chi(2) NR box's E phase beside the tile kernel, 'tb_zchunk' = planes per
        two-step item (an integer; 0 automatic), 'tb_ox' = the most own columns of a two-step
        item (4..124; 0 = 124), 'tb_px' = columns per lane of the two-step kernel (2; 1 = the
        round-5 kernel, kept for A/B), 'tb_pol' = pairs of steps with polarization chunks
        (their general kernel one step at a time beside the rim launches), 'r1_beside' = the
        first rim launch's items other than the narrow strips on a side stream beside the
        two-step kernel, 'tb_lint' = the interior two-step items on a third stream beside the
        previous pair's second rim launch, 'r2_lpt' = the second rim launch in longest-first
        order (the first keeps the narrow strips last), 'strip_zchunk' = planes per narrow
        x-face strip item of the rim (0: the rim's), 'src_guard' = a pair's step sources and
        NaN guard in one launch (mnl_fields_set_schedule)."""
        idx = {"narrow": 0, "dft_pal": 1, "res": 2, "res_tb2": 3, "res_rim": 4, "dft_cmp": 5,
               "rim_zchunk": 6, "nr_early": 7, "tb_zchunk": 8, "tb_ox": 9, "tb_px": 10,
               "tb_pol": 11, "r1_beside": 12, "tb_lint": 13, "r2_lpt": 14,
               "strip_zchunk": 15, "src_guard": 16}[which]
        if idx in (2, 3, 4, 6, 8, 9, 10, 13, 14, 15):  # integers: CUs left free (-1: the default), planes
            check(lib().mnl_fields_set_schedule(self.h, idx, int(value)))
        else:
            check(lib().mnl_fields_set_schedule(self.h, idx, 1 if value else 0))

    def tb_info(self):
        """Temporal blocking of the current fused geometry: dict of
        active (the last call of >= 2 steps stepped in pairs), two-step own cells / border
        points / mixed-palette cells, rim cells / mixed-palette rim cells, item counts, the
        first item's planes, the narrow x-face strip items among the rim items, the
        two-step chunk setting (0: automatic), the most own columns of a two-step item,
        whether polarization chunks step inside the pairs and the interior two-step items (their
        footprint meets no rim box: one rank runs them beside the previous pair's second rim
        launch)."""
        v = (ctypes.c_double * 15)()
        check(lib().mnl_fields_tb_info(self.h, v, 15))
        keys = ("active", "tb_cells", "tb_border", "tb_cells_mixed", "rim_cells",
                "rim_cells_mixed", "tb_items", "rim_items", "tb_planes", "narrow_items", "enabled",
                "tb_zchunk", "tb_width", "tb_pol", "tb_interior_items")
        flags = ("active", "enabled", "tb_pol")
        return {k: (bool(x) if k in flags else int(x)) for k, x in zip(keys, v)}

    def traffic_model(self):
        b = ctypes.c_double()
        c = ctypes.c_double()
        check(lib().mnl_fields_traffic_model(self.h, ctypes.byref(b), ctypes.byref(c)))
        return b.value, c.value


    # -- DFT flux (fields::add_dft_flux, src/dft.cpp:578-640; dft_flux, src/dft.cpp:482-547)
    def dump(self, fname):
        """fields::dump (src/fields_dump.cpp:108-145): t and every per-point state
        array (one file per rank: fname.rank<r> when distributed)."""
        check(lib().mnl_fields_dump(self.h, os.fsencode(fname)))

    def load(self, fname):
        """fields::load (src/fields_dump.cpp:232-270) into fields built the same
        way (structure, sources, flux objects); resumes bit for bit."""
        check(lib().mnl_fields_load(self.h, os.fsencode(fname)))

    def add_dft_flux(self, regions, freqs, decimation=0):
        """regions: [(min xyz, max xyz, direction, weight)]; returns a handle.
        The DFT is accumulated on the GPU after every decimated step."""
        r = np.ascontiguousarray([list(lo) + list(hi) + [d, w] for lo, hi, d, w in regions],
                                 dtype=np.float64).ravel()
        f = np.ascontiguousarray(freqs, dtype=np.float64)
        h = ctypes.c_int()
        check(lib().mnl_fields_add_dft_flux(self.h, len(regions), ptr(r), ptr(f), len(f),
                                            int(decimation), ctypes.byref(h)))
        self._dft_nf = getattr(self, "_dft_nf", {})
        self._dft_nf[h.value] = len(f)
        return h.value

    def flux(self, h):
        """dft_flux::flux (src/dft.cpp:533-547), summed over ranks."""
        out = np.zeros(self._dft_nf[h], dtype=np.float64)
        check(lib().mnl_fields_dft_flux(self.h, h, ptr(out)))
        return out

    def dft_data(self, h, which):
        """DFT values of the E (0) or H (1) chunk list, list order (complex); points
        another rank owns read 0."""
        n = ctypes.c_longlong()
        check(lib().mnl_fields_dft_size(self.h, h, ctypes.byref(n)))
        out = np.zeros(2 * n.value, dtype=np.float64)
        check(lib().mnl_fields_dft_data(self.h, h, int(which), ptr(out), n.value))
        return out[0::2] + 1j * out[1::2]

    def dft_flush(self):
        """Accumulate every buffered DFT update now and wait for the device
        (mnl_fields_dft_flush; readers flush by themselves, updates stay buffered between
        step calls)."""
        check(lib().mnl_fields_dft_flush(self.h))

    def dft_decimation(self, h):
        v = ctypes.c_int()
        check(lib().mnl_fields_dft_decimation(self.h, h, ctypes.byref(v)))
        return v.value

    # -- DFT fields (fields::add_dft_fields / get_dft_array, src/dft.cpp:889-903, 1240-1280)
    def add_dft_fields(self, comps, vmin, vmax, freqs, yee_grid=False, decimation=0):
        """E / H components over [vmin, vmax] on the centered grid (or each
        component's Yee grid); returns a handle (shared with the flux handles)."""
        cs = np.ascontiguousarray(comps, dtype=np.int32)
        lo = np.ascontiguousarray(vmin, dtype=np.float64)
        hi = np.ascontiguousarray(vmax, dtype=np.float64)
        f = np.ascontiguousarray(freqs, dtype=np.float64)
        h = ctypes.c_int()
        check(lib().mnl_fields_add_dft_fields(self.h, len(cs), cs.ctypes.data_as(
            ctypes.POINTER(ctypes.c_int)), ptr(lo), ptr(hi), ptr(f), len(f), int(bool(yee_grid)),
            int(decimation), ctypes.byref(h)))
        self._dft_nf = getattr(self, "_dft_nf", {})
        self._dft_nf[h.value] = len(f)
        return h.value

    def dft_array(self, h, comp, num_freq):
        """fields::get_dft_array(obj, comp, num_freq) for flux and fields handles:
        complex array over the object's volume, empty dimensions collapsed (an empty
        array when the object holds no chunk of comp).  Collective on several ranks."""
        rank = ctypes.c_int()
        dims = (ctypes.c_longlong * 3)()
        check(lib().mnl_fields_dft_array(self.h, h, comp, num_freq, ctypes.byref(rank), dims,
                                         None, 0))
        shape = tuple(dims[k] for k in range(rank.value))
        n = int(np.prod(shape)) if rank.value else 0
        out = np.zeros(2 * max(n, 1), dtype=np.float64)
        check(lib().mnl_fields_dft_array(self.h, h, comp, num_freq, ctypes.byref(rank), dims,
                                         ptr(out), n))
        if not rank.value:
            return np.zeros(0, dtype=np.complex128)
        return (out[0:2 * n:2] + 1j * out[1:2 * n:2]).reshape(shape)


class LocalHub:
    """In-process slab group (mnl_local_hub_create): several z-slabs of one grid on
    one GPU, stepped by one host thread each."""

    def __init__(self, nranks):
        self.h = lib().mnl_local_hub_create(int(nranks))
        self.nranks = nranks

    def __del__(self):
        if getattr(self, "h", None):
            lib().mnl_local_hub_destroy(self.h)
            self.h = None


def device_count():
    n = ctypes.c_int()
    try:
        check(lib().mnl_device_count(ctypes.byref(n)))
    except (RuntimeError, OSError):
        return 0
    return n.value


def slab_range(ncell, rank, nranks):
    lo, hi = ctypes.c_int(), ctypes.c_int()
    check(lib().mnl_slab_range(ncell, rank, nranks, ctypes.byref(lo), ctypes.byref(hi)))
    return lo.value, hi.value


def unique_id():
    """128-byte RCCL unique id (rank 0; broadcast it to the other ranks)."""
    buf = ctypes.create_string_buffer(128)
    check(lib().mnl_comm_unique_id(buf))
    return buf.raw


def ipc_id(nranks):
    """128-byte id of the IPC transport (ranks sharing one GPU): creates the
    shared-memory control block; pass it as nccl_id to every rank's Fields."""
    buf = ctypes.create_string_buffer(128)
    check(lib().mnl_comm_ipc_id(buf, int(nranks)))
    raw = buf.raw
    # rank 0 unlinks the segment once every rank has joined (mnl_comm.cpp init_ipc); if
    # the group never forms (a rank fails before creating its Fields) the creator removes
    # it at exit instead, so nothing stays in /dev/shm
    import atexit

    def _unlink(r=raw):
        try:
            lib().mnl_comm_ipc_unlink(ctypes.create_string_buffer(r, 128))
        except Exception:
            pass
    atexit.register(_unlink)
    return raw


def pick_transport(world, local_rank):
    """Transport and device of one rank: RCCL over xGMI when every local rank has
    its own GPU, the IPC transport when ranks must share one.  Overrides:
    MNL_COMM=rccl|ipc, MNL_BENCH_DEVICE=<device for every rank>.
    Returns (transport, device)."""
    ndev = device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    forced = os.environ.get("MNL_BENCH_DEVICE")
    device = int(forced) if forced else local_rank % max(ndev, 1)
    tr = os.environ.get("MNL_COMM")
    if not tr:
        tr = "ipc" if (forced or ndev < local_world) else "rccl"
    if tr not in ("ipc", "rccl"):
        raise ValueError(f"MNL_COMM must be ipc or rccl, not {tr!r}")
    return tr, device


def comm_id(nranks, transport):
    """Rank-0 side of communicator setup: 'rccl' or 'ipc'."""
    return ipc_id(nranks) if transport == "ipc" else unique_id()


def rccl_selftest(device=0, n=4096):
    """One-rank RCCL send/recv-to-self + allreduce through the slab Comm wrappers."""
    check(lib().mnl_comm_rccl_selftest(int(device), int(n)))


__all__ = ["GridVolume", "Structure", "Fields", "device_count", "unique_id", "ipc_id", "comm_id",
           "math"]
