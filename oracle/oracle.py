"""ctypes wrapper of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
import this module.  The product path (``meep_nl_amd``) never does.

The oracle restates the reference ``fields::step()`` (src/step.cpp:35-140)
chunk by chunk on the CPU; see oracle/mnl_oracle.cpp for the citations.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

# component numbering shared with include/meep_nl_amd.h
Ex, Ey, Ez, Hx, Hy, Hz, Dx, Dy, Dz, Bx, By, Bz = range(12)
X, Y, Z = 0, 1, 2


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        c_int, c_double, c_void = ctypes.c_int, ctypes.c_double, ctypes.c_void_p
        dptr = ctypes.POINTER(ctypes.c_double)
        iptr = ctypes.POINTER(ctypes.c_int)
        L.orc_last_error.restype = ctypes.c_char_p
        L.orc_new.restype = c_void
        L.orc_new.argtypes = [c_int, iptr, c_double, c_double, iptr]
        L.orc_free.argtypes = [c_void]
        L.orc_add_pml.argtypes = [c_void, c_int, c_int, c_double, c_double, c_double]
        L.orc_set_chi1inv.argtypes = [c_void, c_int, c_int, dptr]
        L.orc_set_chi2.argtypes = [c_void, c_int, dptr]
        L.orc_set_chi3.argtypes = [c_void, c_int, dptr]
        L.orc_set_conductivity.argtypes = [c_void, c_int, dptr]
        L.orc_add_custom_point_source.argtypes = [c_void, c_int, SRC_FUNC, ctypes.c_void_p,
                                                  ctypes.c_double, ctypes.c_double, dptr,
                                                  ctypes.c_double, ctypes.c_double, c_int]
        L.orc_array_slice.argtypes = [c_void, c_int, dptr, dptr, c_int, ctypes.POINTER(c_int),
                                      ctypes.POINTER(ctypes.c_longlong), dptr, ctypes.c_longlong]
        L.orc_add_lorentzian_tensor.argtypes = [c_void, ctypes.c_double, ctypes.c_double, c_int,
                                                ctypes.POINTER(dptr)]
        L.orc_add_lorentzian.argtypes = [c_void, c_double, c_double, c_int, dptr, dptr, dptr]
        L.orc_add_susceptibility.argtypes = [c_void, c_int, c_double, c_double, c_int,
                                             ctypes.POINTER(dptr)]
        L.orc_add_point_source.argtypes = [c_void, c_int, c_int, dptr, c_int, dptr, c_double,
                                           c_double, c_int]
        L.orc_require_component.argtypes = [c_void, c_int]
        L.orc_add_volume_source.argtypes = [c_void, c_int, c_int, dptr, c_int, dptr, dptr,
                                            c_double, c_double, c_int, AMP_FUNC, ctypes.c_void_p]
        L.orc_add_custom_volume_source.argtypes = [c_void, c_int, SRC_FUNC, ctypes.c_void_p,
                                                   c_double, c_double, dptr, dptr, c_double,
                                                   c_double, c_int, AMP_FUNC, ctypes.c_void_p]
        L.orc_initialize_field.argtypes = [c_void, c_int, dptr]
        L.orc_energy_in_box.argtypes = [c_void, c_int, dptr, dptr, dptr]
        L.orc_step.argtypes = [c_void, c_int]
        L.orc_get_field.argtypes = [c_void, c_int, dptr, dptr]
        L.orc_copy_component.argtypes = [c_void, c_int, dptr, ctypes.c_size_t]
        L.orc_t.restype = ctypes.c_longlong
        L.orc_t.argtypes = [c_void]
        L.orc_dt.restype = c_double
        L.orc_dt.argtypes = [c_void]
        L.orc_ntot.restype = ctypes.c_size_t
        L.orc_ntot.argtypes = [c_void]
        L.orc_nr_failures.restype = ctypes.c_longlong
        L.orc_nr_failures.argtypes = [c_void]
        L.orc_set_threads.argtypes = [c_int]
        L.orc_set_upstream_nl.argtypes = [c_void, c_int]
        L.orc_add_dft_flux.argtypes = [c_void, c_int, dptr, dptr, c_int, c_int]
        L.orc_dft_flux.argtypes = [c_void, c_int, dptr]
        L.orc_dft_size.restype = ctypes.c_longlong
        L.orc_dft_size.argtypes = [c_void, c_int]
        L.orc_dft_data.argtypes = [c_void, c_int, c_int, dptr, ctypes.c_longlong]
        L.orc_dft_decimation.argtypes = [c_void, c_int]
        L.orc_add_dft_fields.argtypes = [c_void, c_int, iptr, dptr, dptr, dptr, c_int, c_int,
                                         c_int]
        L.orc_dft_array.argtypes = [c_void, c_int, c_int, c_int, iptr,
                                    ctypes.POINTER(ctypes.c_longlong), dptr, ctypes.c_longlong]
        L.orc_eps_average.argtypes = [c_int, iptr, iptr, c_double, c_int, c_int, dptr, c_double,
                                      c_int, c_double, c_int, dptr, dptr, dptr]
        L.orc_sphere_quadrature.argtypes = [c_int, dptr]
        _LIB = L
    return _LIB


SRC_FUNC = ctypes.CFUNCTYPE(None, ctypes.c_double, ctypes.c_void_p,
                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double))
AMP_FUNC = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p,
                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double))


def _chk(rc):
    if rc != 0:
        raise RuntimeError(lib().orc_last_error().decode())


def _dp(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def set_threads(n):
    return lib().orc_set_threads(int(n))


def sphere_quadrature(dim):
    """The restated src/sphere-quad.cpp table for dim 1/2/3: (n, 4) array of
    x, y, z, weight."""
    n = lib().orc_sphere_quadrature(int(dim), None)
    out = np.zeros((n, 4))
    lib().orc_sphere_quadrature(int(dim), _dp(out))
    return out


def eps_average(dim, n, io, a, comp, objs, default_eps=1.0, use_averaging=True, tol=1e-4,
                maxeval=100000):
    """structure_chunk::set_chi1inv with subpixel averaging over geometric objects
    (rows {kind, eps, cx, cy, cz, p0, p1, p2}; src/anisotropic_averaging.cpp:58-298).
    Returns the three rows of E comp `comp` over the canonical grid (1-D: row 0 only)."""
    has = [dim >= 2, dim >= 2, dim != 2]
    shape = tuple(int(n[d]) + 1 for d in range(3) if has[d])
    o = np.ascontiguousarray(np.asarray(objs, dtype=np.float64).reshape(-1, 8))
    rows = [np.zeros(shape) for _ in range(3)]
    if dim == 1:
        rows[1] = rows[2] = None
    na = (ctypes.c_int * 3)(*[int(v) for v in n])
    ia = (ctypes.c_int * 3)(*[int(v) for v in io])
    _chk(lib().orc_eps_average(int(dim), na, ia, float(a), int(comp), o.shape[0], _dp(o),
                               float(default_eps), int(bool(use_averaging)), float(tol),
                               int(maxeval), *[_dp(r) for r in rows]))
    return rows


class Oracle:
    """One oracle simulation on a Meep-style grid_volume.

    ``dim`` 1 uses the Z direction only (Meep's D1), 2 uses X,Y, 3 uses X,Y,Z.
    ``io`` is the little corner in half-pixel units (0 = Meep default origin,
    ``-n`` per direction = ``center_origin()`` for even n).
    """

    def __init__(self, dim, n, a, courant=0.5, io=(0, 0, 0)):
        self.dim = dim
        self.n = [int(v) for v in n]
        self.a = float(a)
        self.io = [int(v) for v in io]
        na = (ctypes.c_int * 3)(*self.n)
        ia = (ctypes.c_int * 3)(*self.io)
        self.h = lib().orc_new(dim, na, self.a, float(courant), ia)
        if not self.h:
            raise RuntimeError(lib().orc_last_error().decode())
        self.has = [dim >= 2, dim >= 2, dim != 2]

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_free(self.h)
            self.h = None

    # ---- geometry helpers (canonical layout: Z fastest, n+1 points per present dir)
    def shape(self):
        return tuple(self.n[d] + 1 for d in range(3) if self.has[d])

    def shift(self, c, d):
        if not self.has[d]:
            return 0
        t = c // 3
        if t in (0, 2):
            return 1 if d == c % 3 else 0
        return 1 if d != c % 3 else 0

    def coords(self, c):
        """Positions (in length units) of every array point of component c."""
        axes = []
        for d in range(3):
            if self.has[d]:
                j = np.arange(self.n[d] + 1)
                axes.append((self.io[d] + 2 * j + self.shift(c, d)) * (0.5 / self.a))
        return np.meshgrid(*axes, indexing="ij")

    # ---- structure
    def add_pml(self, thickness, dirs=(0, 1, 2), sides=(0, 1), R=1e-15, mean_stretch=1.0):
        for d in dirs:
            for s in sides:
                _chk(lib().orc_add_pml(self.h, d, s, thickness, R, mean_stretch))

    def set_chi1inv(self, comp, d, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64).ravel()
        self._keep = getattr(self, "_keep", []) + [arr]
        _chk(lib().orc_set_chi1inv(self.h, comp, d, _dp(arr)))

    def set_epsilon_fn(self, fn):
        """Non-averaged epsilon (eps_averaging=False): chi1inv = 1/eps(loc)."""
        for c in (Ex, Ey, Ez):
            if self.dim == 1 and c != Ex:
                continue
            pts = self.coords(c)
            self.set_chi1inv(c, c % 3, 1.0 / fn(*pts))

    def set_epsilon_geometry(self, objs, default_eps=1.0, use_averaging=True, tol=1e-4,
                             maxeval=100000):
        """structure::set_epsilon(material_function &, use_anisotropic_averaging, tol,
        maxeval) over geometric objects: every E component's rows from eps_average,
        trivial off-diagonal rows (and all-trivial tensors) dropped."""
        for c in ((Ex,) if self.dim == 1 else (Ex, Ey, Ez)):
            rows = eps_average(self.dim, self.n, self.io, self.a, c, objs, default_eps,
                               use_averaging, tol, maxeval)
            triv = [r is None or np.all(r == (1.0 if d == c else 0.0)) for d, r in enumerate(rows)]
            for d, r in enumerate(rows):
                if r is None or (d != c and triv[d]) or all(triv):
                    continue
                self.set_chi1inv(c, d, r)

    def set_chi2(self, comp, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64).ravel()
        _chk(lib().orc_set_chi2(self.h, comp, _dp(arr)))

    def set_chi3(self, comp, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64).ravel()
        _chk(lib().orc_set_chi3(self.h, comp, _dp(arr)))

    def set_conductivity(self, comp, arr):
        """structure::set_conductivity (src/structure.cpp:868-905); D/B (or E/H)
        component, None = zero."""
        a = None if arr is None else np.ascontiguousarray(arr, dtype=np.float64).ravel()
        _chk(lib().orc_set_conductivity(self.h, comp, None if a is None else _dp(a)))

    def add_lorentzian_tensor(self, omega0, gamma, sigma, drude=False):
        arrs = [None if sigma[c][d] is None else
                np.ascontiguousarray(sigma[c][d], dtype=np.float64).ravel()
                for c in range(3) for d in range(3)]
        ptrs = (ctypes.POINTER(ctypes.c_double) * 9)(*[_dp(a) if a is not None else None for a in arrs])
        _chk(lib().orc_add_lorentzian_tensor(self.h, omega0, gamma, int(drude), ptrs))

    def get_array_slice(self, comp, vmin, vmax, snap=False):
        """fields::get_array_slice over the volume [vmin, vmax] (3 coordinates, unused
        ones ignored); shape = the kept (non-empty) directions in X, Y, Z order."""
        lo = np.ascontiguousarray(vmin, dtype=np.float64)
        hi = np.ascontiguousarray(vmax, dtype=np.float64)
        rank = ctypes.c_int(0)
        dims = (ctypes.c_longlong * 3)()
        _chk(lib().orc_array_slice(self.h, comp, _dp(lo), _dp(hi), int(snap), ctypes.byref(rank), dims,
                                   None, 0))
        shape = tuple(dims[k] for k in range(rank.value))
        out = np.zeros(int(np.prod(shape)) if shape else 1)
        _chk(lib().orc_array_slice(self.h, comp, _dp(lo), _dp(hi), int(snap), ctypes.byref(rank),
                                   dims, _dp(out), out.size))
        return out.reshape(shape) if shape else out[0]

    def add_custom_source(self, comp, func, start, end, pos, amp=1.0, is_integrated=False):
        cbs = self.__dict__.setdefault("_custom_cbs", {})
        if id(func) not in cbs:
            def _cb(t, _data, re, im, func=func):
                v = complex(func(t))
                re[0] = v.real
                im[0] = v.imag
            cbs[id(func)] = (func, SRC_FUNC(_cb))
        p = np.ascontiguousarray(list(pos) + [0.0] * (3 - len(pos)), dtype=np.float64)
        a = complex(amp)
        _chk(lib().orc_add_custom_point_source(self.h, comp, cbs[id(func)][1], None, float(start),
                                               float(end), _dp(p), a.real, a.imag,
                                               int(is_integrated)))

    def add_lorentzian(self, omega0, gamma, sigmas, drude=False):
        s = [None if v is None else np.ascontiguousarray(v, dtype=np.float64).ravel()
             for v in sigmas]
        _chk(lib().orc_add_lorentzian(self.h, omega0, gamma, int(drude), *[_dp(v) for v in s]))

    def add_magnetic_lorentzian(self, omega0, gamma, sigmas, drude=False):
        """add_susceptibility(sigma, H_stuff, lorentzian): diagonal sigma at the H
        components' points (None = 0)."""
        arrs = [None] * 9
        for d in range(3):
            if sigmas[d] is not None:
                arrs[4 * d] = np.ascontiguousarray(sigmas[d], dtype=np.float64).ravel()
        self._keep = getattr(self, "_keep", []) + [a for a in arrs if a is not None]
        ptrs = (ctypes.POINTER(ctypes.c_double) * 9)(*[_dp(a) if a is not None else None for a in arrs])
        _chk(lib().orc_add_susceptibility(self.h, 1, omega0, gamma, int(drude), ptrs))

    def set_mu_fn(self, fn):
        """Non-averaged mu: chi1inv of the H components = 1/mu(loc) (set_mu)."""
        for c in (Hx, Hy, Hz):
            if self.dim == 1 and c != Hy:
                continue
            pts = self.coords(c)
            self.set_chi1inv(c, c % 3, 1.0 / fn(*pts))

    # ---- fields
    def add_point_source(self, comp, kind, params, pos, amp=1.0, is_integrated=False):
        p = np.ascontiguousarray(params, dtype=np.float64)
        pos = np.ascontiguousarray(list(pos) + [0.0] * (3 - len(pos)), dtype=np.float64)
        amp = complex(amp)
        _chk(lib().orc_add_point_source(self.h, comp, kind, _dp(p), len(p), _dp(pos), amp.real,
                                        amp.imag, int(is_integrated)))

    def _amp_cb(self, amp_func):
        if amp_func is None:
            return AMP_FUNC()
        def _cb(rel, _data, re, im, f=amp_func):
            v = complex(f((rel[0], rel[1], rel[2])))
            re[0] = v.real
            im[0] = v.imag
        cb = AMP_FUNC(_cb)
        self.__dict__.setdefault("_amp_cbs", []).append(cb)
        return cb

    def add_volume_source(self, comp, kind, params, vmin, vmax, amp=1.0, is_integrated=False,
                          amp_func=None):
        """fields::add_volume_source (src/sources.cpp:455-494)."""
        p = np.ascontiguousarray(params, dtype=np.float64)
        lo = np.ascontiguousarray(list(vmin) + [0.0] * (3 - len(vmin)), dtype=np.float64)
        hi = np.ascontiguousarray(list(vmax) + [0.0] * (3 - len(vmax)), dtype=np.float64)
        a = complex(amp)
        _chk(lib().orc_add_volume_source(self.h, comp, kind, _dp(p), len(p), _dp(lo), _dp(hi),
                                         a.real, a.imag, int(is_integrated),
                                         self._amp_cb(amp_func), None))

    def add_custom_volume_source(self, comp, func, start, end, vmin, vmax, amp=1.0,
                                 is_integrated=False, amp_func=None):
        cbs = self.__dict__.setdefault("_custom_cbs", {})
        if id(func) not in cbs:
            def _cb(t, _data, re, im, func=func):
                v = complex(func(t))
                re[0] = v.real
                im[0] = v.imag
            cbs[id(func)] = (func, SRC_FUNC(_cb))
        lo = np.ascontiguousarray(list(vmin) + [0.0] * (3 - len(vmin)), dtype=np.float64)
        hi = np.ascontiguousarray(list(vmax) + [0.0] * (3 - len(vmax)), dtype=np.float64)
        a = complex(amp)
        _chk(lib().orc_add_custom_volume_source(self.h, comp, cbs[id(func)][1], None, float(start),
                                                float(end), _dp(lo), _dp(hi), a.real, a.imag,
                                                int(is_integrated), self._amp_cb(amp_func), None))

    def add_gaussian_volume_source(self, comp, freq, width, start, end, vmin, vmax, amp=1.0,
                                   is_integrated=False, amp_func=None):
        self.add_volume_source(comp, 0, [freq, width, start, end], vmin, vmax, amp, is_integrated,
                               amp_func)

    def add_gaussian_source(self, comp, freq, width, start, end, pos, amp=1.0,
                            is_integrated=False):
        self.add_point_source(comp, 0, [freq, width, start, end], pos, amp, is_integrated)

    def add_continuous_source(self, comp, freq, width, start, end, slowness, pos, amp=1.0,
                              is_integrated=False):
        f = complex(freq)
        self.add_point_source(comp, 1, [f.real, f.imag, width, start, end, slowness], pos, amp,
                              is_integrated)

    def legacy_point_source(self, comp, freq, width, peaktime, cutoff, pos, amp):
        """fields::add_point_source(c, freq, width, peaktime, cutoff, vec, amp) -- the
        deprecated C++ form used by tests/known_results.cpp (src/sources.cpp:189-211).
        C++ src_time default is_integrated=true (src/meep.hpp:950-951)."""
        width = width / freq
        dt = self.dt
        cutoff = (1.0 / self.a) + cutoff * width
        if peaktime <= 0.0:
            peaktime = self.t * dt + cutoff
        peaktime += (-dt * 0.5) if comp in (Hx, Hy, Hz) else dt
        self.add_gaussian_source(comp, freq, width, peaktime - cutoff, peaktime + cutoff, pos, amp,
                                 is_integrated=comp not in (Hx, Hy, Hz))

    def require_component(self, comp):
        _chk(lib().orc_require_component(self.h, comp))

    def initialize_field(self, comp, values):
        """fields::initialize_field (src/initialize.cpp:135-161); values: whole-cell
        array (or callable over coords(comp)), real part."""
        if callable(values):
            values = values(*self.coords(comp))
        v = np.ascontiguousarray(np.real(np.broadcast_to(values, self.shape())),
                                 dtype=np.float64).ravel()
        _chk(lib().orc_initialize_field(self.h, comp, _dp(v)))

    def step(self, n=1):
        _chk(lib().orc_step(self.h, int(n)))

    def _energy(self, which, vmin=None, vmax=None):
        out = ctypes.c_double()
        lo = None if vmin is None else np.ascontiguousarray(vmin, dtype=np.float64)
        hi = None if vmax is None else np.ascontiguousarray(vmax, dtype=np.float64)
        _chk(lib().orc_energy_in_box(self.h, which, _dp(lo), _dp(hi), ctypes.byref(out)))
        return out.value

    def electric_energy_in_box(self, vmin=None, vmax=None):
        return self._energy(0, vmin, vmax)

    def magnetic_energy_in_box(self, vmin=None, vmax=None):
        return self._energy(1, vmin, vmax)

    def field_energy_in_box(self, vmin=None, vmax=None):
        return self._energy(2, vmin, vmax)

    def field_energy(self):
        """fields::field_energy (src/energy_and_flux.cpp:48): the whole cell."""
        return self._energy(2)

    @property
    def t(self):
        return lib().orc_t(self.h)

    @property
    def dt(self):
        return lib().orc_dt(self.h)

    def time(self):
        return self.t * self.dt

    def round_time(self):
        return float(np.float32(self.t * self.dt))

    def get_field(self, comp, pos):
        pos = np.ascontiguousarray(list(pos) + [0.0] * (3 - len(pos)), dtype=np.float64)
        out = ctypes.c_double()
        _chk(lib().orc_get_field(self.h, comp, _dp(pos), ctypes.byref(out)))
        return out.value

    def get_array(self, comp):
        nt = lib().orc_ntot(self.h)
        out = np.zeros(nt, dtype=np.float64)
        _chk(lib().orc_copy_component(self.h, comp, _dp(out), nt))
        return out.reshape(self.shape())

    def nr_random_fallbacks(self):
        return lib().orc_nr_failures(self.h)

    def set_upstream_nl(self, on=True):
        """Upstream Meep chi2/chi3 (Pade approximant) instead of the fork's NR /
        inert chi3."""
        _chk(lib().orc_set_upstream_nl(self.h, int(on)))

    # ---- DFT flux (fields::add_dft_flux, src/dft.cpp:578-640)
    def add_dft_flux(self, regions, freqs, decimation=0):
        """regions: [(min xyz, max xyz, direction, weight)]; returns a handle."""
        r = np.ascontiguousarray([list(lo) + list(hi) + [d, w] for lo, hi, d, w in regions],
                                 dtype=np.float64).ravel()
        f = np.ascontiguousarray(freqs, dtype=np.float64)
        h = lib().orc_add_dft_flux(self.h, len(regions), _dp(r), _dp(f), len(f), int(decimation))
        if h < 0:
            raise RuntimeError(lib().orc_last_error().decode())
        self._dft_nf = getattr(self, "_dft_nf", {})
        self._dft_nf[h] = len(f)
        return h

    def flux(self, h):
        out = np.zeros(self._dft_nf[h], dtype=np.float64)
        _chk(lib().orc_dft_flux(self.h, h, _dp(out)))
        return out

    def dft_data(self, h, which):
        """All DFT values of the E (0) or H (1) chunk list, in list order (complex)."""
        n = lib().orc_dft_size(self.h, h)
        out = np.zeros(2 * n, dtype=np.float64)
        _chk(lib().orc_dft_data(self.h, h, int(which), _dp(out), n))
        return out[0::2] + 1j * out[1::2]

    def dft_decimation(self, h):
        return lib().orc_dft_decimation(self.h, h)

    # ---- DFT fields (fields::add_dft_fields / get_dft_array, src/dft.cpp:889-903, 1240-1280)
    def add_dft_fields(self, comps, vmin, vmax, freqs, yee_grid=False, decimation=0):
        cs = np.ascontiguousarray(comps, dtype=np.int32)
        lo = np.ascontiguousarray(vmin, dtype=np.float64)
        hi = np.ascontiguousarray(vmax, dtype=np.float64)
        f = np.ascontiguousarray(freqs, dtype=np.float64)
        h = lib().orc_add_dft_fields(self.h, len(cs), cs.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                     _dp(lo), _dp(hi), _dp(f), len(f), int(bool(yee_grid)),
                                     int(decimation))
        if h < 0:
            raise RuntimeError(lib().orc_last_error().decode())
        self._dft_nf = getattr(self, "_dft_nf", {})
        self._dft_nf[h] = len(f)
        return h

    def dft_array(self, h, comp, num_freq):
        """get_dft_array(obj, comp, num_freq): complex array, empty dimensions collapsed."""
        rank = ctypes.c_int(0)
        dims = (ctypes.c_longlong * 3)()
        _chk(lib().orc_dft_array(self.h, h, comp, num_freq, ctypes.byref(rank), dims, None, 0))
        shape = tuple(dims[k] for k in range(rank.value))
        if not rank.value:  # no chunk of comp (process_dft_component: rank 0, no array)
            return np.zeros(0, dtype=np.complex128)
        n = int(np.prod(shape))
        out = np.zeros(2 * max(n, 1), dtype=np.float64)
        _chk(lib().orc_dft_array(self.h, h, comp, num_freq, ctypes.byref(rank), dims, _dp(out), n))
        return (out[0:2 * n:2] + 1j * out[1:2 * n:2]).reshape(shape)

    def center(self):
        """grid_volume::center() (src/vec.cpp:1089-1103): io + round_down_to_even(n)."""
        out = []
        for d in range(3):
            if self.has[d]:
                n = self.n[d] - (self.n[d] & 1)
                out.append((self.io[d] + n) * (0.5 / self.a))
            else:
                out.append(0.0)
        return out


def meep_vol(dim, sizes, a, center_origin=False, courant=0.5):
    """vol1d/vol2d/vol3d (src/vec.cpp:904-931) [+ center_origin]."""
    n = [0, 0, 0]
    if dim == 1:
        n[2] = int(sizes[0] * a + 0.5)
    elif dim == 2:
        n[0] = 1 if sizes[0] == 0 else int(sizes[0] * a + 0.5)
        n[1] = 1 if sizes[1] == 0 else int(sizes[1] * a + 0.5)
    else:
        n = [1 if s == 0 else int(s * a + 0.5) for s in sizes]
    io = [0, 0, 0]
    if center_origin:
        io = [-(v - (v & 1)) for v in n]
    return Oracle(dim, n, a, courant, io)
