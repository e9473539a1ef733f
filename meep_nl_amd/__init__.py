"""meep_nl_amd -- MI355X-native fields::step() hot path of PMack10/meep_nl.

``meep_nl_amd.Simulation`` mirrors the meep.Simulation subset that drives the
time stepper; ``meep_nl_amd.core`` mirrors the C++ structure/fields API.
Both call libmnl.so (HIP kernels for gfx950 + C-ABI, include/meep_nl_amd.h).
"""
from .core import (Bx, By, Bz, Dielectric, Dx, Dy, Dz, Ex, Ey, Ez, Fields, GridVolume, Hx, Hy,
                   Hz, Permeability, Structure, X, Y, Z, device_count)
from .simulation import (ALL, AUTOMATIC, Block, ContinuousSource, CustomSource, Cylinder,
                         DftFields, DftFlux, Sphere,
                         DrudeSusceptibility,
                         FluxRegion, GaussianSource, High, LorentzianSusceptibility, Low, Medium,
                         PML, Simulation, Source, Vector3, Volume, after_sources, after_time,
                         air, at_beginning, at_end, at_every, before_time, combine_step_funcs,
                         during_sources, get_flux_freqs, get_fluxes, inf, stop_after_walltime,
                         stop_when_fields_decayed, vacuum, when_false, when_true, verbosity,
                         quiet, wall_time)

__version__ = "0.1.0"
