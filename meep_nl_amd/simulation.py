"""Python drop-in for the meep.Simulation subset that drives fields::step().

Mirrors python/simulation.py (Simulation.__init__ 1228-1256, init_sim
2449-2512, _run_until 2795-2855, round_time/meep_time 2609-2636) and
python/source.py (Source.add_source 132-158, GaussianSource 262-332,
ContinuousSource) for Cartesian 1-D/2-D/3-D cells with real fields, PML,
non-averaged block geometry (epsilon, chi2, chi3, Lorentzian/Drude E
susceptibilities) and point sources.  Everything runs on the MI355X through
libmnl.so; there is no CPU path.
"""
import inspect
import math
import numbers
import os
import time
import warnings

import numpy as np

from . import core
from .core import Bx, By, Bz, Dielectric, Dx, Dy, Dz, Ex, Ey, Ez, Hx, Hy, Hz, Permeability, X, Y, Z

ALL = -1
Low, High = 0, 1
inf = 1.0e20


class Vector3:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)

    def __iter__(self):
        return iter((self.x, self.y, self.z))

    def __getitem__(self, i):
        return (self.x, self.y, self.z)[i]

    def __add__(self, o):
        return Vector3(self.x + o[0], self.y + o[1], self.z + o[2])

    def __sub__(self, o):
        return Vector3(self.x - o[0], self.y - o[1], self.z - o[2])

    def __mul__(self, s):
        return Vector3(self.x * s, self.y * s, self.z * s)

    __rmul__ = __mul__

    def __eq__(self, o):
        return tuple(self) == tuple(o)

    def __repr__(self):
        return f"Vector3({self.x}, {self.y}, {self.z})"


class Volume:
    def __init__(self, center=Vector3(), size=Vector3()):
        self.center = Vector3(*center)
        self.size = Vector3(*size)


# ---------------------------------------------------------------- materials
class LorentzianSusceptibility:
    """lorentzian_susceptibility(frequency, gamma) with constant sigma
    (python/geom.py LorentzianSusceptibility; src/susceptibility.cpp:188-262)."""

    drude = False

    def __init__(self, frequency=0.0, gamma=0.0, sigma=1.0, sigma_diag=None, sigma_offdiag=None):
        self.frequency = float(frequency)
        self.gamma = float(gamma)
        sd = sigma_diag if sigma_diag is not None else Vector3(sigma, sigma, sigma)
        self.sigma_diag = Vector3(*sd)
        # (xy, xz, yz) of the symmetric sigma tensor (python/geom.py:717-737)
        self.sigma_offdiag = Vector3(*(sigma_offdiag if sigma_offdiag is not None else (0, 0, 0)))

    def sigma_row(self, c):
        """Row c of the sigma tensor [[a, u, v], [u, b, w], [v, w, c]]."""
        dg, od = self.sigma_diag, self.sigma_offdiag
        t = [[dg.x, od.x, od.y], [od.x, dg.y, od.z], [od.y, od.z, dg.z]]
        return t[c]

    def key(self):
        return (self.frequency, self.gamma, self.drude)


class DrudeSusceptibility(LorentzianSusceptibility):
    drude = True


class Medium:
    def __init__(self, epsilon=1.0, epsilon_diag=None, epsilon_offdiag=None, E_chi2=0.0,
                 E_chi3=0.0, chi2=None, chi3=None, E_susceptibilities=(), index=None, mu=1.0,
                 D_conductivity=None, B_conductivity=None, D_conductivity_diag=None,
                 B_conductivity_diag=None, mu_diag=None, mu_offdiag=None,
                 H_susceptibilities=()):
        if index is not None:
            epsilon = index * index
        self.epsilon_diag = Vector3(*(epsilon_diag if epsilon_diag is not None else
                                      (epsilon, epsilon, epsilon)))
        self.epsilon_offdiag = Vector3(*(epsilon_offdiag if epsilon_offdiag is not None else
                                         (0, 0, 0)))
        self.E_chi2 = float(chi2 if chi2 is not None else E_chi2)
        self.E_chi3 = float(chi3 if chi3 is not None else E_chi3)
        self.E_susceptibilities = list(E_susceptibilities)
        # python/geom.py Medium: a scalar *_conductivity sets the whole diagonal
        self.D_conductivity_diag = Vector3(*(D_conductivity_diag if D_conductivity_diag is not None
                                             else (D_conductivity or 0.0,) * 3))
        self.B_conductivity_diag = Vector3(*(B_conductivity_diag if B_conductivity_diag is not None
                                             else (B_conductivity or 0.0,) * 3))
        # permeability (python/geom.py Medium: mu_diag / mu_offdiag = (xy, xz, yz)) and
        # magnetic susceptibilities (H_susceptibilities; diagonal sigma only here)
        self.mu_diag = Vector3(*(mu_diag if mu_diag is not None else (mu, mu, mu)))
        self.mu_offdiag = Vector3(*(mu_offdiag if mu_offdiag is not None else (0, 0, 0)))
        self.H_susceptibilities = list(H_susceptibilities)
        for su in self.H_susceptibilities:
            if su.sigma_offdiag != Vector3():
                raise NotImplementedError("magnetic susceptibilities: diagonal sigma only")


vacuum = air = Medium()


class Block:
    def __init__(self, size=Vector3(), center=Vector3(), material=Medium(), **kw):
        self.size = Vector3(*size)
        self.center = Vector3(*center)
        self.material = material
        if any(k in kw for k in ("e1", "e2", "e3")):
            raise NotImplementedError("only axis-aligned blocks are supported")

    def contains(self, x, y, z):
        c, s = self.center, self.size
        return ((np.abs(x - c.x) <= 0.5 * s.x) & (np.abs(y - c.y) <= 0.5 * s.y) &
                (np.abs(z - c.z) <= 0.5 * s.z))

    def geo_record(self, eps):
        """Row of mnl_structure_set_epsilon_geometry (kind 0 = block)."""
        c, s = self.center, self.size
        return [0, eps, c.x, c.y, c.z, s.x, s.y, s.z]


class Sphere:
    """meep.Sphere (python/geom.py): |r - center| <= radius."""

    def __init__(self, radius, center=Vector3(), material=Medium(), **kw):
        self.radius = float(radius)
        self.center = Vector3(*center)
        self.material = material

    def contains(self, x, y, z):
        c = self.center
        dx, dy, dz = x - c.x, y - c.y, z - c.z
        return dx * dx + dy * dy + dz * dz <= self.radius * self.radius

    def geo_record(self, eps):
        c = self.center
        return [1, eps, c.x, c.y, c.z, self.radius, 0.0, 0.0]


class Cylinder:
    """meep.Cylinder (python/geom.py) with its axis along x, y or z."""

    def __init__(self, radius, height=1e20, axis=Vector3(0, 0, 1), center=Vector3(),
                 material=Medium(), **kw):
        self.radius = float(radius)
        self.height = float(height)
        self.center = Vector3(*center)
        self.material = material
        ax = [abs(v) for v in Vector3(*axis)]
        if sorted(ax) != [0.0, 0.0, max(ax)] or max(ax) == 0:
            raise NotImplementedError("only cylinders along x, y or z are supported")
        self.axis = ax.index(max(ax))

    def contains(self, x, y, z):
        c = self.center
        d = [x - c.x, y - c.y, z - c.z]
        a = d[self.axis]
        u, v = [d[k] for k in range(3) if k != self.axis]
        return (np.abs(a) <= 0.5 * self.height) & (u * u + v * v <= self.radius * self.radius)

    def geo_record(self, eps):
        c = self.center
        return [2, eps, c.x, c.y, c.z, self.radius, self.height, float(self.axis)]


class PML:
    def __init__(self, thickness, direction=ALL, side=ALL, R_asymptotic=1e-15, mean_stretch=1.0):
        self.thickness = float(thickness)
        self.direction = direction
        self.side = side
        self.R_asymptotic = R_asymptotic
        self.mean_stretch = mean_stretch


# ---------------------------------------------------------------- sources
class SourceTime:
    is_integrated = False


class GaussianSource(SourceTime):
    """python/source.py:262-332 -> gaussian_src_time(f, w, start, start+2w*cutoff)."""

    def __init__(self, frequency=None, width=0, fwidth=float("inf"), start_time=0, cutoff=5.0,
                 is_integrated=False, wavelength=None):
        if frequency is None and wavelength is None:
            raise ValueError("Must set either frequency or wavelength in GaussianSource.")
        self.frequency = 1 / wavelength if wavelength else float(frequency)
        self.width = max(width, 1 / fwidth)
        self.start_time = start_time
        self.cutoff = cutoff
        self.is_integrated = is_integrated

    def params(self):
        return 0, [self.frequency, self.width, self.start_time,
                   self.start_time + 2 * self.width * self.cutoff]


class ContinuousSource(SourceTime):
    def __init__(self, frequency=None, start_time=0, end_time=inf, width=0, fwidth=float("inf"),
                 slowness=3.0, is_integrated=False, wavelength=None):
        if frequency is None and wavelength is None:
            raise ValueError("Must set either frequency or wavelength in ContinuousSource.")
        self.frequency = 1 / wavelength if wavelength else frequency
        self.start_time, self.end_time = start_time, end_time
        self.width = max(width, 1 / fwidth)
        self.slowness = slowness
        self.is_integrated = is_integrated

    def params(self):
        f = complex(self.frequency)
        return 1, [f.real, f.imag, self.width, self.start_time, self.end_time, self.slowness]


class CustomSource(SourceTime):
    """python/source.py:338-400 -> custom_src_time(src_func, start, end, f, fw):
    src_func(t) is the (complex) dipole, or the current if not is_integrated."""

    def __init__(self, src_func, start_time=-1.0e20, end_time=1.0e20, is_integrated=False,
                 center_frequency=0, fwidth=0):
        self.src_func = src_func
        self.start_time, self.end_time = start_time, end_time
        self.is_integrated = is_integrated
        self.center_frequency, self.fwidth = center_frequency, fwidth
        self.frequency = center_frequency


class Source:
    """python/source.py:22-158: a current source over the volume (center, size) --
    a point, line, plane or box -- with an optional amplitude function
    amp_func(Vector3 relative to the center) -> complex."""

    def __init__(self, src, component, center=None, volume=None, size=Vector3(), amplitude=1.0,
                 amp_func=None, amp_func_file=None, amp_data=None):
        if center is None and volume is None:
            raise ValueError("Source requires either center or volume")
        self.src = src
        self.component = component
        if volume is not None:
            center, size = volume.center, volume.size
        self.center = Vector3(*center)
        self.size = Vector3(*size)
        self.amplitude = complex(amplitude)
        self.amp_func = amp_func
        self.amp_data = None if amp_data is None else np.asarray(amp_data, dtype=np.complex128)
        if amp_func_file is not None:
            raise NotImplementedError("amp_func_file (HDF5 amplitude profiles): no HDF5 in this "
                                      "build; pass the array as amp_data")

    def _amp_data_func(self):
        """amp_file_func (src/sources.cpp:347-374): the array linearly interpolated
        over the source volume (map_coordinates / linear_interpolate,
        src/fields.cpp:767-825, mirror boundaries)."""
        a = self.amp_data
        while a.ndim < 3:
            a = a[..., None]
        nx, ny, nz = a.shape
        re, im = np.ascontiguousarray(a.real).ravel(), np.ascontiguousarray(a.imag).ravel()
        size = self.size

        def mirror(i, n):
            return 2 * n - 1 - i if i >= n else (-1 - i if i < 0 else i)

        def coords(r, n):
            r = -r if r < 0.0 else (1.0 - r if r > 1.0 else r)
            i1 = mirror(int(r * n), n)
            d = r * n - i1 - 0.5
            i2 = mirror(i1 + 1 if d >= 0.0 else i1 - 1, n)
            return i1, i2, abs(d)

        def interp(data, rx, ry, rz):
            x1, x2, dx = coords(rx, nx)
            y1, y2, dy = coords(ry, ny)
            z1, z2, dz = coords(rz, nz)

            def D(x, y, z):
                return data[(x * ny + y) * nz + z]
            return (((D(x1, y1, z1) * (1.0 - dx) + D(x2, y1, z1) * dx) * (1.0 - dy) +
                     (D(x1, y2, z1) * (1.0 - dx) + D(x2, y2, z1) * dx) * dy) * (1.0 - dz) +
                    ((D(x1, y1, z2) * (1.0 - dx) + D(x2, y1, z2) * dx) * (1.0 - dy) +
                     (D(x1, y2, z2) * (1.0 - dx) + D(x2, y2, z2) * dx) * dy) * dz)

        def f(p):
            r = [0.0 if size[d] == 0 else 0.5 + p[d] / size[d] for d in range(3)]
            return complex(interp(re, *r), interp(im, *r))
        return f

    def add_source(self, fields):  # python/source.py:132-158 -> fields::add_volume_source
        lo = tuple(c - 0.5 * s for c, s in zip(self.center, self.size))
        hi = tuple(c + 0.5 * s for c, s in zip(self.center, self.size))
        af = None
        if self.amp_func is not None:
            af = (lambda f: lambda r: f(Vector3(*r)))(self.amp_func)
        elif self.amp_data is not None:
            af = self._amp_data_func()
        if isinstance(self.src, CustomSource):
            fields.add_custom_volume_source(self.component, self.src.src_func, self.src.start_time,
                                            self.src.end_time, lo, hi, self.amplitude,
                                            self.src.is_integrated, af)
            return
        kind, p = self.src.params()
        fields.add_volume_source(self.component, kind, p, lo, hi, self.amplitude,
                                 self.src.is_integrated, af)


# ---------------------------------------------------------------- flux monitors
AUTOMATIC = -1


def fix_dft_args(args, i):
    """(fcen, df, nfreq) -> frequency list (python/simulation.py:72-93)."""
    if (len(args) > i + 2 and isinstance(args[i], (int, float))
            and isinstance(args[i + 1], (int, float)) and isinstance(args[i + 2], int)):
        fcen, df, nfreq = args[i], args[i + 1], args[i + 2]
        freq = [fcen] if nfreq == 1 else np.linspace(fcen - 0.5 * df, fcen + 0.5 * df, nfreq)
        return args[:i] + (freq,) + args[i + 3:]
    if not isinstance(args[i], (np.ndarray, list, tuple)):
        raise TypeError("add_dft functions only accept fcen,df,nfreq (3 numbers) or freq "
                        "(array/list)")
    return args


class FluxRegion:
    """python/simulation.py:510-570: a plane/line/point/volume and a flux direction."""

    def __init__(self, center=None, size=Vector3(), direction=AUTOMATIC, weight=1.0,
                 volume=None):
        if center is None and volume is None:
            raise ValueError("Either center or volume required")
        if volume is not None:
            center, size = volume.center, volume.size
        self.center = Vector3(*center)
        self.size = Vector3(*size)
        self.direction = direction
        self.weight = complex(weight)


def _normal_direction(dim, size):
    """volume::normal_direction (src/vec.cpp:227-262) for Cartesian cells."""
    if dim == 1:
        return Z
    if dim == 2:
        if size.x == 0 and size.y > 0:
            return X
        if size.x > 0 and size.y == 0:
            return Y
        # fields::normal_direction pads empty dims (src/dft.cpp:791-809): no further case in 2-D
        raise RuntimeError("Could not determine normal direction for given grid_volume.")
    zero = [size.x == 0, size.y == 0, size.z == 0]
    if sum(zero) == 1:
        return zero.index(True)
    raise RuntimeError("Could not determine normal direction for given grid_volume.")


class DftFlux:
    """python/simulation.py:687-760 (flux object); the DFT lives on the GPU."""

    def __init__(self, sim, freq, regions, decimation_factor):
        self.sim = sim
        self.freq = [float(f) for f in freq]
        self.regions = list(regions)
        self.decimation_factor = decimation_factor
        self.handle = None

    def _create(self):
        sim = self.sim
        regs = []
        for r in self.regions:
            if r.weight.imag != 0:
                raise NotImplementedError("complex flux weights are out of scope (real fields)")
            d = _normal_direction(sim.dimensions, r.size) if r.direction < 0 else r.direction
            lo = [r.center[k] - 0.5 * r.size[k] for k in range(3)]
            hi = [r.center[k] + 0.5 * r.size[k] for k in range(3)]
            if sim.dimensions == 1:  # 1-D cells live on the z axis
                lo, hi = [0.0, 0.0, lo[2]], [0.0, 0.0, hi[2]]
            elif sim.dimensions == 2:
                lo[2] = hi[2] = 0.0
            regs.append((lo, hi, d, r.weight.real))
        self.handle = sim.fields.add_dft_flux(regs, self.freq, self.decimation_factor)

    def flux(self):
        return list(self.sim.fields.flux(self.handle))


class DftFields:
    """python/simulation.py:793-810 (dft_fields object, created by add_dft_fields);
    the DFT lives on the GPU."""

    def __init__(self, sim, components, freq, lo, hi, yee_grid, decimation_factor):
        self.sim = sim
        self.components = [int(c) for c in components]
        self.freq = [float(f) for f in freq]
        self.lo, self.hi = lo, hi
        self.yee_grid = bool(yee_grid)
        self.decimation_factor = int(decimation_factor)
        self.handle = None

    def _create(self):
        self.handle = self.sim.fields.add_dft_fields(self.components, self.lo, self.hi, self.freq,
                                                     self.yee_grid, self.decimation_factor)


def get_flux_freqs(f):
    """python/simulation.py:6014-6019"""
    return list(f.freq)


def get_fluxes(f):
    """python/simulation.py:6022-6027"""
    return f.flux()


# ---------------------------------------------------------------- step functions
def _num_args(func):
    code = getattr(func, "__code__", None)
    if code is None:
        return 1
    n = code.co_argcount
    return n - 1 if inspect.ismethod(func) else n


def _eval_step_func(sim, func, todo):
    """python/simulation.py:4999-5008"""
    n = _num_args(func)
    if n == 1:
        if todo == "step":
            func(sim)
    elif n == 2:
        func(sim, todo)
    else:
        raise ValueError(f"Step function '{func.__name__}' requires 1 or 2 arguments")


def _when_true_funcs(cond, *step_funcs):
    def _true(sim, todo):
        if todo == "finish" or cond(sim):
            for f in step_funcs:
                _eval_step_func(sim, f, todo)
    return _true


def after_sources(*step_funcs):
    """python/simulation.py:5023-5035"""
    def _after_sources(sim, todo):
        if sim.round_time() >= sim.fields.last_source_time():
            for f in step_funcs:
                _eval_step_func(sim, f, todo)
    return _after_sources


def after_time(t, *step_funcs):
    return _when_true_funcs(lambda sim: sim.round_time() >= t, *step_funcs)


def before_time(t, *step_funcs):
    return _when_true_funcs(lambda sim: sim.round_time() < t, *step_funcs)


def when_true(cond, *step_funcs):
    return _when_true_funcs(cond, *step_funcs)


def when_false(cond, *step_funcs):
    return _when_true_funcs(lambda sim: not cond(sim), *step_funcs)


def at_beginning(*step_funcs):
    closure = {"done": False}

    def _beg(sim, todo):
        if not closure["done"]:
            for f in step_funcs:
                _eval_step_func(sim, f, todo)
            closure["done"] = True
    return _beg


def at_end(*step_funcs):
    def _end(sim, todo):
        if todo == "finish":
            for f in step_funcs:
                _eval_step_func(sim, f, "step")
            for f in step_funcs:
                _eval_step_func(sim, f, "finish")
    return _end


def at_every(dt, *step_funcs):
    """python/simulation.py:5096-5110"""
    closure = {"tlast": 0.0}

    def _every(sim, todo):
        t = sim.round_time()
        if todo == "finish" or t >= closure["tlast"] + dt + (-0.5 * sim.fields.dt):
            for f in step_funcs:
                _eval_step_func(sim, f, todo)
            closure["tlast"] = t
    return _every


def during_sources(*step_funcs):
    closure = {"finished": False}

    def _during(sim, todo):
        if sim.round_time() < sim.fields.last_source_time():
            for f in step_funcs:
                _eval_step_func(sim, f, "step")
        elif not closure["finished"]:
            for f in step_funcs:
                _eval_step_func(sim, f, "finish")
            closure["finished"] = True
    return _during


def combine_step_funcs(*step_funcs):
    def _combine(sim, todo):
        for f in step_funcs:
            _eval_step_func(sim, f, todo)
    return _combine


def stop_when_fields_decayed(dt=None, c=None, pt=None, decay_by=None):
    """python/simulation.py:5225-5273: every dt time units compare the maximum
    |c(pt)|^2 of the last interval with the maximum so far."""
    if dt is None or c is None or pt is None or decay_by is None:
        raise ValueError("dt, c, pt, and decay_by are all required.")
    closure = {"max_abs": 0, "cur_max": 0, "t0": 0}

    def _stop(sim):
        v = sim.get_field_point(c, pt)
        fabs = abs(v) * abs(v)
        closure["cur_max"] = max(closure["cur_max"], fabs)
        if sim.round_time() <= dt + closure["t0"]:
            return False
        old_cur = closure["cur_max"]
        closure["cur_max"] = 0
        closure["t0"] = sim.round_time()
        closure["max_abs"] = max(closure["max_abs"], old_cur)
        return old_cur <= closure["max_abs"] * decay_by
    return _stop


def stop_after_walltime(t):
    start = time.time()
    return lambda sim: time.time() - start > t


# ---------------------------------------------------------------- distributed
def _dist_context():
    """(rank, world, device, comm_id) when launched one process per GPU by
    torch.distributed.run, else None.  The transport is RCCL when every local
    rank has its own GPU, the IPC transport when ranks share one
    (core.pick_transport)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    rank = dist.get_rank()
    transport, device = core.pick_transport(world, int(os.environ.get("LOCAL_RANK", rank)))
    obj = [core.comm_id(world, transport) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return rank, world, device, obj[0]


def _dist_barrier():
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.barrier()


# ---------------------------------------------------------------- verbosity
class Verbosity:
    """meep.verbosity (python/verbosity_mgr.py): one process-wide level, 0 quiet,
    1 progress messages (default), 2 more; `verbosity(2)` or `verbosity.meep = 2`
    sets it, also for the native library's "on time step" lines."""
    _instance = None

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
            cls._instance._level = 1
        return cls._instance

    def get(self):
        return self._level

    def set(self, level):
        self._level = int(level)
        try:
            core.set_verbosity(self._level)
        except Exception:  # native library absent: the level still applies here
            pass
        return self._level

    def __call__(self, level=None):
        return self.get() if level is None else self.set(level)

    @property
    def meep(self):
        return self._level

    @meep.setter
    def meep(self, level):
        self.set(level)

    def __int__(self):
        return self._level

    def __repr__(self):
        return f"Verbosity: level={self._level}"


verbosity = Verbosity()


def quiet(quietval=True):
    """meep.quiet: verbosity 0 (or back to 1)."""
    verbosity(0 if quietval else 1)


def wall_time():
    return time.time()


def _progress(t0, t, dt):
    """display_progress (python/simulation.py:5468-5489): every dt seconds of wall
    time, "Meep progress: ..." while running until t0 + t."""
    start = time.time()
    last = {"t": start}

    def show(sim):
        now = time.time()
        if now - last["t"] < dt:
            return
        done = sim.meep_time() - t0
        pct = done / (0.01 * t)
        el = now - start
        togo = (el * (t / done) - el) if done != 0 else 0
        if verbosity.meep > 0 and sim._is_master():
            print("Meep progress: {}/{} = {:.1f}% done in {:.1f}s, {:.1f}s to go".format(
                done, t, pct, el, togo))
        last["t"] = now
    return show


# ---------------------------------------------------------------- Simulation
_WARNED_AVERAGING = False


class Simulation:
    def __init__(self, cell_size, resolution, geometry=(), sources=(), boundary_layers=(),
                 default_material=Medium(), Courant=0.5, eps_averaging=True, dimensions=None,
                 force_complex_fields=False, k_point=False, symmetries=(), parallel=None,
                 nonlinear_mode="fork", progress_interval=4, time_phases=True, **kwargs):
        self.cell_size = Vector3(*cell_size)
        self.resolution = float(resolution)
        self.geometry = list(geometry)
        self.sources = list(sources)
        self.boundary_layers = list(boundary_layers)
        self.default_material = default_material
        self.Courant = float(Courant)
        self.eps_averaging = eps_averaging
        self.subpixel_tol = float(kwargs.pop("subpixel_tol", 1e-4))
        self.subpixel_maxeval = int(kwargs.pop("subpixel_maxeval", 100000))
        if force_complex_fields or k_point or symmetries:
            raise NotImplementedError("complex fields / Bloch k_point / symmetries are out of scope")
        if dimensions is None:
            dimensions = 3 if self.cell_size.z != 0 else 2
            if self.cell_size.x == 0 and self.cell_size.y == 0:
                dimensions = 1
        self.dimensions = dimensions
        self.parallel = parallel
        # "upstream": Meep's Pade chi2/chi3 E update instead of the fork's (an
        # extension; the fork's behaviour is the default)
        self.nonlinear_mode = nonlinear_mode
        self.progress_interval = progress_interval
        # per-phase GPU times (HIP events) for print_times / time_spent_on; False skips
        # the event records (bench.py --no-events measures their cost: about 0.3 % of a
        # fused 512^3 step, profiles/README.md)
        self.time_phases = bool(time_phases)
        self.run_index = 0
        self.fields = None
        self.structure = None
        self.dft_objects = []

    # -- structure
    def _create_grid_volume(self):
        sz = self.cell_size
        sizes = [sz.z] if self.dimensions == 1 else ([sz.x, sz.y] if self.dimensions == 2
                                                     else [sz.x, sz.y, sz.z])
        return core.GridVolume.vol(self.dimensions, sizes, self.resolution, center_origin=True)

    def _materials_at(self, gv, c, offset=(0.0, 0.0, 0.0)):
        """Per-point material of component c (no subpixel averaging), optionally at
        the Yee points shifted by `offset`."""
        pts = gv.coords(c)
        full = [np.zeros(gv.shape()) for _ in range(3)]
        k = 0
        for d in range(3):
            if gv.has[d]:
                full[d] = pts[k] + offset[d]
                k += 1
        idx = np.full(gv.shape(), -1, dtype=np.int32)
        for i, g in enumerate(self.geometry):
            idx[g.contains(*full)] = i
        mats = [self.default_material] + [g.material for g in self.geometry]
        return idx + 1, mats

    def _init_structure(self, device=-1):
        gv = self._create_grid_volume()
        s = core.Structure(gv, self.Courant)
        if self.nonlinear_mode != "fork":
            s.set_nonlinear_mode(self.nonlinear_mode)
        for layer in self.boundary_layers:
            if not isinstance(layer, PML):
                raise NotImplementedError("only PML boundary layers are supported")
            dirs = (0, 1, 2) if layer.direction == ALL else (layer.direction,)
            sides = (0, 1) if layer.side == ALL else (layer.side,)
            s.add_pml(layer.thickness, dirs, sides, layer.R_asymptotic, layer.mean_stretch)
        media = [self.default_material] + [g.material for g in self.geometry]
        uniform = len(self.geometry) == 0
        need_eps = any(m.epsilon_diag != Vector3(1, 1, 1) or m.epsilon_offdiag != Vector3()
                       for m in media)
        # subpixel averaging (structure::set_epsilon with anisotropic averaging, the C++
        # core's material_function algorithm, src/anisotropic_averaging.cpp:58-298) on the
        # device, for media of isotropic permittivity; Python Meep's libctl averaging
        # (meepgeom.cpp) is not available, see DESIGN.md
        iso = all(m.epsilon_diag.x == m.epsilon_diag.y == m.epsilon_diag.z and
                  m.epsilon_offdiag == Vector3() for m in media)
        averaged = False
        if self.eps_averaging and not uniform and need_eps:
            if iso:
                global _WARNED_AVERAGING
                if not _WARNED_AVERAGING:
                    _WARNED_AVERAGING = True
                    warnings.warn(
                        "eps_averaging: subpixel averaging follows the C++ core's "
                        "material_function algorithm (src/anisotropic_averaging.cpp), not "
                        "Python Meep's libctl averaging (meepgeom.cpp), so epsilon near "
                        "interfaces differs from Python Meep at the averaging tolerance "
                        "(parity unpinned: no reference value covers it, DESIGN.md section 22)",
                        RuntimeWarning)
                s.set_epsilon_geometry([g.geo_record(g.material.epsilon_diag.x)
                                        for g in self.geometry],
                                       default_eps=self.default_material.epsilon_diag.x,
                                       use_anisotropic_averaging=True,
                                       tol=self.subpixel_tol, maxeval=self.subpixel_maxeval,
                                       device=device)
                averaged = True
            else:
                warnings.warn("eps_averaging over anisotropic media is not implemented; "
                              "materials are sampled at the Yee points", RuntimeWarning)
        need_chi2 = any(m.E_chi2 != 0 for m in media)
        need_chi3 = any(m.E_chi3 != 0 for m in media)
        sus_keys = []
        for m in media:
            for su in m.E_susceptibilities:
                if su.key() not in sus_keys:
                    sus_keys.append(su.key())
        comps = (Ex,) if self.dimensions == 1 else (Ex, Ey, Ez)
        sus_sig = {k: [[None] * 3 for _ in range(3)] for k in sus_keys}
        for c in comps:
            d = c % 3
            which, mats = self._materials_at(gv, c)
            def table(f):
                return np.array([f(m) for m in mats], dtype=np.float64)[which]
            if need_eps and not averaged:
                # chi1inv row of the inverse permittivity tensor of each medium
                # (Medium.epsilon_diag / epsilon_offdiag = (xy, xz, yz)); the fork only
                # uses the diagonal value and whether off-diagonal entries are zero.
                inv = []
                for m in mats:
                    e, o = m.epsilon_diag, m.epsilon_offdiag
                    T = np.array([[e.x, o.x, o.y], [o.x, e.y, o.z], [o.y, o.z, e.z]])
                    inv.append(np.linalg.inv(T) if any(v != 0 for v in o) else
                               np.diag([1.0 / e.x, 1.0 / e.y, 1.0 / e.z]))
                inv = np.array(inv)
                s.set_chi1inv(c, d, inv[:, d, d][which])
                if any(m.epsilon_offdiag != Vector3() for m in mats):
                    for k in (1, 2):
                        dd = (d + k) % 3
                        s.set_chi1inv(c, dd, inv[:, d, dd][which])
            if need_chi3:
                s.set_chi3(c, table(lambda m: m.E_chi3))
            if need_chi2:
                s.set_chi2(c, table(lambda m: m.E_chi2))
            for key in sus_keys:
                def sig(m, key=key, row=d, col=d):
                    for su in m.E_susceptibilities:
                        if su.key() == key:
                            return su.sigma_row(row)[col]
                    return 0.0
                sus_sig[key][d][d] = table(sig)
                if any(su.sigma_offdiag != Vector3() for m in mats for su in m.E_susceptibilities
                       if su.key() == key):
                    # off-diagonal entries sampled half a pixel back along d
                    # (src/anisotropic_averaging.cpp:334-341)
                    h = [0.0, 0.0, 0.0]
                    h[d] = -0.5 / self.resolution
                    which_o, mats_o = self._materials_at(gv, c, offset=h)
                    for col in range(3):
                        if col != d and self.dimensions != 1:
                            sus_sig[key][d][col] = np.array(
                                [sig(m, col=col) for m in mats_o], dtype=np.float64)[which_o]
        for key in sus_keys:
            s.add_lorentzian_tensor(key[0], key[1], sus_sig[key], drude=key[2])
        self._init_h_materials(gv, s, media)
        # structure::set_materials -> set_conductivity(c, mat) for the D and B
        # components with nonzero conductivity (src/structure.cpp:378-380, 868-905),
        # sampled at each component's own Yee points
        for attr, base in (("D_conductivity_diag", Dx), ("B_conductivity_diag", Bx)):
            if not any(getattr(m, attr) != Vector3() for m in media):
                continue
            for d in ((0,) if base == Dx else (1,)) if self.dimensions == 1 else (0, 1, 2):
                c = base + d
                which, mats = self._materials_at(gv, c)
                s.set_conductivity(c, np.array([getattr(m, attr)[d] for m in mats],
                                               dtype=np.float64)[which])
        self.structure = s
        return s

    def _init_h_materials(self, gv, s, media):
        """structure::set_mu (chi1inv of the H components, sampled at the H Yee points:
        no subpixel averaging of mu here) and add_susceptibility(sigma, H_stuff, ...) for
        the media's H_susceptibilities (src/anisotropic_averaging.cpp:221-372)."""
        need_mu = any(m.mu_diag != Vector3(1, 1, 1) or m.mu_offdiag != Vector3() for m in media)
        hkeys = []
        for m in media:
            for su in m.H_susceptibilities:
                if su.key() not in hkeys:
                    hkeys.append(su.key())
        if not need_mu and not hkeys:
            return
        if need_mu and self.eps_averaging and len(self.geometry) > 0:
            warnings.warn("mu is sampled at the H Yee points (no subpixel averaging of mu)",
                          RuntimeWarning)
        comps = (Hy,) if self.dimensions == 1 else (Hx, Hy, Hz)
        hsig = {k: [None, None, None] for k in hkeys}
        for c in comps:
            d = c % 3
            which, mats = self._materials_at(gv, c)
            if need_mu:
                inv = []
                for m in mats:
                    e, o = m.mu_diag, m.mu_offdiag
                    T = np.array([[e.x, o.x, o.y], [o.x, e.y, o.z], [o.y, o.z, e.z]])
                    inv.append(np.linalg.inv(T) if any(v != 0 for v in o) else
                               np.diag([1.0 / e.x, 1.0 / e.y, 1.0 / e.z]))
                inv = np.array(inv)
                s.set_chi1inv(c, d, inv[:, d, d][which])
                if any(m.mu_offdiag != Vector3() for m in mats):
                    for k in (1, 2):
                        s.set_chi1inv(c, (d + k) % 3, inv[:, d, (d + k) % 3][which])
            for key in hkeys:
                def sig(m, key=key, row=d):
                    for su in m.H_susceptibilities:
                        if su.key() == key:
                            return su.sigma_row(row)[row]
                    return 0.0
                hsig[key][d] = np.array([sig(m) for m in mats], dtype=np.float64)[which]
        for key in hkeys:
            s.add_magnetic_lorentzian(key[0], key[1], hsig[key], drude=key[2])

    def has_mu(self):
        """Simulation.has_mu (python/simulation.py): some medium has mu != 1."""
        media = [self.default_material] + [g.material for g in self.geometry]
        return any(m.mu_diag != Vector3(1, 1, 1) or m.mu_offdiag != Vector3() for m in media)

    def init_sim(self):
        if self.fields is not None:
            return
        ctx = _dist_context() if self.parallel is not False else None
        if self.structure is None:
            self._init_structure(device=ctx[2] if ctx else -1)
        if ctx:
            rank, world, local, nid = ctx
            self.fields = core.Fields(self.structure, device=local, rank=rank, nranks=world,
                                      nccl_id=nid)
        else:
            self.fields = core.Fields(self.structure)
        # per-phase GPU times for print_times (HIP events; ~0.3 % of a step)
        self.fields.set_profiling(self.time_phases)
        for src in self.sources:
            src.add_source(self.fields)
        if getattr(self, "load_fields_file", None):  # delayed load (python/simulation.py:2509-2510)
            self.load_fields(self.load_fields_file)

    def initialize_field(self, cmpnt=None, amp_func=None):
        """Simulation.initialize_field (python/simulation.py:2520-2532) ->
        fields::initialize_field (src/initialize.cpp:135-161): amp_func(Vector3)
        -> complex at every point of the component (real part kept)."""
        self.init_sim()
        gv = self.fields.gv
        pts = [p.ravel() for p in gv.coords(cmpnt)]
        full = [np.zeros(pts[0].size) for _ in range(3)]
        k = 0
        for d in range(3):
            if gv.has[d]:
                full[d] = pts[k]
                k += 1
        vals = np.array([complex(amp_func(Vector3(x, y, z))).real
                         for x, y, z in zip(*full)], dtype=np.float64)
        self.fields.initialize_field(cmpnt, vals.reshape(gv.shape()))

    # -- time
    def meep_time(self):
        self.init_sim()
        return self.fields.time()

    def round_time(self):
        self.init_sim()
        return self.fields.round_time()

    @property
    def timestep(self):
        self.init_sim()
        return self.fields.t

    # -- running
    def run(self, *step_funcs, until=None, until_after_sources=None):
        """Simulation.run (python/simulation.py:4502-4540): until= a time, a condition
        function or a list of them; until_after_sources= the same, counted from the
        end of the sources (_run_sources_until, 2857-2876)."""
        self.init_sim()
        if until_after_sources is not None:
            self._run_sources_until(until_after_sources, step_funcs)
        elif until is not None:
            self._run_until(until, step_funcs)
        else:
            raise ValueError("Invalid run configuration")

    def _run_until(self, cond, step_funcs):
        """python/simulation.py:2795-2855: stop when any condition holds; a number T
        means round_time() >= t0 + T.  Step functions run before every step, once
        more after the loop, then with 'finish'."""
        self.init_sim()
        conds = list(cond) if isinstance(cond, (list, tuple)) else [cond]
        step_funcs = list(step_funcs)
        t0 = self.round_time()
        if not step_funcs and all(isinstance(c, numbers.Number) for c in conds):
            # every condition is a time: count the steps on the host, step in
            # batches (one call each; a progress message between batches)
            stop = t0 + min(conds)
            t, dt = self.fields._time()
            n = 0
            while float(np.float32((t + n) * dt)) < stop:
                n += 1
            show = _progress(t0, min(conds), self.progress_interval)
            batch = 64
            while n > 0:
                m = min(n, batch)
                w = time.time()
                self.fields.step(m)
                n -= m
                show(self)
                if time.time() - w < 0.25:
                    batch *= 2
            self._run_finished()
            return
        for i, c in enumerate(conds):
            if isinstance(c, numbers.Number):
                step_funcs.append(_progress(t0, c, self.progress_interval))
                conds[i] = (lambda T: lambda sim: sim.round_time() >= t0 + T)(c)
            elif not callable(c):
                raise TypeError(f"Stopping condition {c} is not a number or a function")
        while not any(c(self) for c in conds):
            for fn in step_funcs:
                _eval_step_func(self, fn, "step")
            self.fields.step(1)
        for fn in step_funcs:
            _eval_step_func(self, fn, "step")
        for fn in step_funcs:
            _eval_step_func(self, fn, "finish")
        self._run_finished()

    def _is_master(self):
        return self.fields is None or self.fields.rank == 0

    def _run_finished(self):
        if verbosity.meep > 0 and self._is_master():
            print("run {} finished at t = {} ({} timesteps)".format(
                self.run_index, self.meep_time(), self.fields.t))
        self.run_index += 1

    # -- timing (python/simulation.py:4542-4601 -> src/time.cpp:130-215)
    def _times_all(self):
        """Per-process seconds, shape (n_sinks, nprocs) (timing_data_vector_from_all)."""
        self.init_sim()
        n = self.fields.nranks
        mine = self.fields.time_spent()
        allt = np.zeros((len(core.TIME_SINKS), n))
        allt[:, self.fields.rank] = mine
        return self.fields.sum_to_all(allt.ravel()).reshape(allt.shape)

    def print_times(self):
        """fields::print_times: mean (and stddev over processes) of each time sink."""
        if self.fields is None:
            return
        allt = self._times_all()
        n = allt.shape[1]
        if not self._is_master():
            return
        print("\nField time usage:")
        for (_, label), row in zip(core.TIME_SINKS, allt):
            mean = float(np.sum(row)) / n
            var = float(np.sum(row * row)) - n * mean * mean
            sd = 0.0 if (n == 1 or var <= 0) else math.sqrt(var / (n - 1))
            if mean != 0:
                if sd != 0:
                    print("    %21s: %4.6g s +/- %4.6g s" % (label, mean, sd))
                else:
                    print("    %21s: %4.6g s" % (label, mean))
        print()
        if verbosity.meep > 1:
            print("\nField time usage for all processes:")
            for (_, label), row in zip(core.TIME_SINKS, allt):
                print("    %21s: " % label + ", ".join("%4.6g" % v for v in row))
            print()

    def time_spent_on(self, time_sink):
        """Seconds each process spent on time_sink (meep::time_sink enum value)."""
        return self._times_all()[int(time_sink)].tolist()

    def mean_time_spent_on(self, time_sink):
        t = self.time_spent_on(time_sink)
        return sum(t) / len(t)

    def get_timing_data(self):
        allt = self._times_all()
        return {k: allt[k].tolist() for k in range(allt.shape[0])}

    def output_times(self, fname):
        """fields::output_times: CSV, one header row of sink labels, one row per process."""
        if self.fields is None:
            return
        if not fname.endswith(".csv"):
            fname += ".csv"
        allt = self._times_all()
        if not self._is_master():
            return
        if verbosity.meep > 0:
            print('outputting timing statistics to file "%s"...' % fname)
        with open(fname, "w") as fh:
            fh.write(", ".join(label for _, label in core.TIME_SINKS) + "\n")
            for j in range(allt.shape[1]):
                fh.write(", ".join("%g" % v for v in allt[:, j]) + "\n")

    def _run_sources_until(self, cond, step_funcs):
        self.init_sim()
        conds = list(cond) if isinstance(cond, (list, tuple)) else [cond]
        ts = self.fields.last_source_time()
        new = []
        for c in conds:
            if isinstance(c, numbers.Number):
                new.append((ts - self.round_time()) + c)
            else:
                new.append((lambda f: lambda sim: f(sim) and sim.round_time() >= ts)(c))
        self._run_until(new, step_funcs)

    # -- flux spectra
    def add_flux(self, *args, **kwargs):
        """add_flux(fcen, df, nfreq, *FluxRegions) or add_flux(freq, *FluxRegions)
        (python/simulation.py:3470-3505); initialises the fields first."""
        args = fix_dft_args(args, 0)
        freq, regions = args[0], args[1:]
        flux = DftFlux(self, freq, regions, kwargs.get("decimation_factor", 0))
        self.init_sim()
        flux._create()
        self.dft_objects.append(flux)
        return flux

    def _where_bounds(self, where=None, center=None, size=None):
        """_volume_from_kwargs (python/simulation.py:2253-2262): where, else center +
        size, else the whole grid volume (fields::total_volume)."""
        if where is not None:
            center, size = where.center, where.size
        dirs = (2,) if self.dimensions == 1 else ((0, 1) if self.dimensions == 2 else (0, 1, 2))
        lo, hi = [0.0] * 3, [0.0] * 3
        if center is None or size is None:
            gv = self.structure.gv
            for d in dirs:
                lo[d] = gv.io[d] * (0.5 / gv.a)
                hi[d] = (gv.io[d] + 2 * gv.n[d]) * (0.5 / gv.a)
            return lo, hi
        center, size = Vector3(*center), Vector3(*size)
        for d in dirs:
            lo[d] = center[d] - 0.5 * size[d]
            hi[d] = center[d] + 0.5 * size[d]
        return lo, hi

    def add_dft_fields(self, *args, **kwargs):
        """add_dft_fields(cs, fcen, df, nfreq | freq, where=None, center=None, size=None,
        yee_grid=False, decimation_factor=0) (python/simulation.py:2976-3036) ->
        fields::add_dft_fields (src/dft.cpp:889-903); initialises the fields first."""
        components = list(args[0])
        args = fix_dft_args(args, 1)
        freq = args[1]
        self.init_sim()
        lo, hi = self._where_bounds(kwargs.get("where"), kwargs.get("center"), kwargs.get("size"))
        if kwargs.get("persist", False):
            pass  # persist only keeps chunks across a structure change (not modelled here)
        dftf = DftFields(self, components, freq, lo, hi, kwargs.get("yee_grid", False),
                         kwargs.get("decimation_factor", 0))
        dftf._create()
        self.dft_objects.append(dftf)
        return dftf

    def get_dft_array(self, dft_obj=None, component=None, num_freq=None):
        """Simulation.get_dft_array (python/simulation.py:3988-4026) for dft_fields and
        dft_flux objects -> fields::get_dft_array (src/dft.cpp:1240-1280): a complex
        array over the object's volume (empty dimensions collapsed)."""
        if not self.dft_objects:
            raise RuntimeError("DFT monitor dft_obj must be initialized before calling "
                               "get_dft_array")
        if not isinstance(dft_obj, (DftFields, DftFlux)):
            raise ValueError(f"Invalid type of dft object: {dft_obj}")
        return self.fields.dft_array(dft_obj.handle, int(component), int(num_freq))

    # -- checkpoint (python/simulation.py:2293-2450); flat binary files, not HDF5
    def _load_dump_dirname(self, dirname, single_parallel_file=True):
        if single_parallel_file:
            return dirname
        ctx = _dist_context() if self.parallel is not False else None
        return os.path.join(dirname, "rank%02d" % (ctx[0] if ctx else 0))

    def dump_structure(self, fname, single_parallel_file=True):
        if self.structure is None:
            raise ValueError("Structure must be initialized before calling dump_structure")
        self.structure.dump(fname)

    def load_structure(self, fname, single_parallel_file=True):
        if self.structure is None:
            raise ValueError("Structure must be initialized before loading structure from file "
                             "'%s'" % fname)
        if self.fields is not None:
            raise ValueError("load_structure must be called before the fields are created")
        self.structure.load(fname)

    def dump_fields(self, fname, single_parallel_file=True):
        if self.fields is None:
            raise ValueError("Fields must be initialized before calling dump_fields")
        self.fields.dump(fname)

    def load_fields(self, fname, single_parallel_file=True):
        if self.fields is None:
            raise ValueError("Fields must be initialized before loading fields from file '%s'"
                             % fname)
        self.fields.load(fname)

    def dump(self, dirname, dump_structure=True, dump_fields=True, single_parallel_file=True):
        d = self._load_dump_dirname(dirname, single_parallel_file)
        os.makedirs(d, exist_ok=True)
        if dump_structure:
            # the structure description is global: with a single parallel file only
            # the master writes it (structure::dump, src/structure_dump.cpp), and no
            # rank returns before it is complete
            rank = self.fields.rank if self.fields is not None else 0
            if not single_parallel_file or rank == 0:
                self.dump_structure(os.path.join(d, "structure.mnl"))
            if single_parallel_file:
                _dist_barrier()
        if dump_fields:
            self.dump_fields(os.path.join(d, "fields.mnl"))

    def load(self, dirname, load_structure=True, load_fields=True, single_parallel_file=True):
        """Call right after creating the Simulation, before init_sim (as the
        reference): the structure is loaded when it is built, the fields after
        the sources are added."""
        d = self._load_dump_dirname(dirname, single_parallel_file)
        if load_structure:
            if self.structure is None:
                self._init_structure()
            self.load_structure(os.path.join(d, "structure.mnl"))
        if load_fields:
            f = os.path.join(d, "fields.mnl")
            if self.fields is not None:
                self.load_fields(f)
            else:
                self.load_fields_file = f

    # -- monitors
    def get_field_point(self, c, pt):
        self.init_sim()
        return self.fields.get_field(c, tuple(pt))

    def get_array(self, component=Ez, vol=None, center=None, size=None, cmplx=None, arr=None,
                  frequency=0, snap=False):
        """Simulation.get_array (python/simulation.py:3872-3990) ->
        fields::get_array_slice over the volume (default: the whole cell) on the
        Centered grid, empty dimensions interpolated and collapsed.  Real fields
        only; snap=True snaps empty dimensions to the nearest grid point."""
        self.init_sim()
        if cmplx or frequency:
            raise NotImplementedError("get_array: complex / frequency-dependent slices")
        if vol is not None:
            center, size = vol.center, vol.size
        center = Vector3(*(center if center is not None else Vector3()))
        size = Vector3(*(size if size is not None else self.cell_size))
        lo, hi = [0.0] * 3, [0.0] * 3
        dirs = (2,) if self.dimensions == 1 else ((0, 1) if self.dimensions == 2 else (0, 1, 2))
        for d in dirs:
            lo[d] = center[d] - 0.5 * size[d]
            hi[d] = center[d] + 0.5 * size[d]
        out = self.fields.get_array_slice(component, lo, hi, snap)
        if arr is not None:
            arr[...] = out
            return arr
        return out

    def get_epsilon(self, frequency=0, snap=False):
        """Simulation.get_epsilon (python/simulation.py:4603-4604) = get_array(Dielectric):
        epsilon on the Centered grid from the diagonal chi1inv (src/array_slice.cpp:385-396)."""
        return self.get_array(component=Dielectric, frequency=frequency, snap=snap)

    def get_mu(self, frequency=0, snap=False):
        """Simulation.get_mu = get_array(Permeability) (src/array_slice.cpp:397-408)."""
        return self.get_array(component=Permeability, frequency=frequency, snap=snap)

    def change_sources(self, new_sources):
        """Simulation.change_sources (python/simulation.py:4454-4463): replace the
        sources, in the running fields too (fields::remove_sources + add_source)."""
        self.sources = list(new_sources)
        if self.fields is not None:
            self.fields.remove_sources()
            for src in self.sources:
                src.add_source(self.fields)

    def restart_fields(self):
        """Simulation.restart_fields (python/simulation.py:4479-4490): time 0, zero
        fields (fields::zero_fields); the Fourier transforms keep accumulating."""
        if self.fields is not None:
            self.fields.t = 0
            self.fields.zero_fields()
        else:
            self.init_sim()

    def reset_meep(self):
        """Simulation.reset_meep (python/simulation.py:4465-4477): drop fields, structure
        and DFT objects."""
        self.fields = None
        self.structure = None
        self.dft_objects = []

    def _energy(self, which, box, center, size):
        if self.fields is None:
            raise RuntimeError(f"Fields must be initialized before using {which}")
        lo, hi = self._where_bounds(box, center, size)
        return getattr(self.fields, which)(lo, hi)

    def electric_energy_in_box(self, box=None, center=None, size=None):
        """python/simulation.py:3655-3674 -> fields::electric_energy_in_box."""
        return self._energy("electric_energy_in_box", box, center, size)

    def magnetic_energy_in_box(self, box=None, center=None, size=None):
        """python/simulation.py:3676-3695 -> fields::magnetic_energy_in_box."""
        return self._energy("magnetic_energy_in_box", box, center, size)

    def field_energy_in_box(self, box=None, center=None, size=None):
        """python/simulation.py:3697-3716 -> fields::field_energy_in_box."""
        return self._energy("field_energy_in_box", box, center, size)

    def get_component_array(self, component=Ez):
        """The raw whole-cell array of a component (Yee layout, ghosts 0)."""
        self.init_sim()
        return self.fields.get_array(component)
