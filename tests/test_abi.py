"""CPU checks of the C-ABI boundary: the library loads, exports every symbol
include/meep_nl_amd.h declares, host-only calls work, and the product path
fails loudly (no CPU fallback) when there is no HIP device."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def libpath():
    path = os.path.join(ROOT, "meep_nl_amd", "libmnl.so")
    if not os.path.exists(path):
        subprocess.run(["bash", os.path.join(ROOT, "meep_nl_amd", "csrc", "build.sh")], check=True)
    return path


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "meep_nl_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mnl_[a-z_0-9]+)\s*\(", txt)))


def test_exports_every_header_symbol(libpath):
    out = subprocess.run(["nm", "-D", "--defined-only", libpath], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (mnl_\w+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    from meep_nl_amd import _lib
    assert set(_lib.exported_symbols()) == set(header_symbols())


def test_structure_host_calls(libpath):
    from meep_nl_amd import core
    gv = core.GridVolume.vol(3, [1.0, 1.2, 0.8], 10, center_origin=True)
    assert gv.shape() == (11, 13, 9)
    s = core.Structure(gv)
    s.add_pml(0.3)
    s.set_chi1inv(0, 0, np.full(gv.shape(), 0.5))
    s.set_chi2(0, np.zeros(gv.shape()))
    s.add_lorentzian(1.0, 0.1, [np.ones(gv.shape()), None, None])
    s.set_box(0, [-0.1, 0.1, -0.1, 0.1, -0.1, 0.1], 4.0)
    s.set_chi1inv(5, 2, np.full(gv.shape(), 0.25))  # mu of Hz (set_mu)
    assert np.array_equal(s.get_chi1inv(5, 2), np.full(gv.shape(), 0.25))
    s.add_magnetic_lorentzian(1.0, 0.1, [None, np.ones(gv.shape()), None])
    with pytest.raises(RuntimeError):
        s.set_chi1inv(8, 0, np.ones(gv.shape()))  # D has no chi1inv


def test_errors_are_meep_aborts(libpath):
    from meep_nl_amd import core
    with pytest.raises(RuntimeError, match="meep:"):
        core.Structure(core.GridVolume(3, [1, 4, 4], 10))


def test_no_cpu_fallback(libpath):
    from meep_nl_amd import core
    if core.device_count() > 0:
        pytest.skip("GPU present")
    s = core.Structure(core.GridVolume.vol(2, [1, 1], 10))
    with pytest.raises(RuntimeError, match="no HIP device"):
        core.Fields(s)


def test_simulation_setup_host_side(libpath):
    import meep_nl_amd as mp
    sim = mp.Simulation(
        cell_size=mp.Vector3(2, 2, 2), resolution=8, eps_averaging=False,
        boundary_layers=[mp.PML(0.5)],
        geometry=[mp.Block(size=mp.Vector3(mp.inf, 1, 1),
                           material=mp.Medium(epsilon=12, E_chi3=1e-2,
                                              E_susceptibilities=[mp.LorentzianSusceptibility(
                                                  1.1, 0.05, 0.5)]))],
        sources=[mp.Source(mp.GaussianSource(0.15, fwidth=0.1), mp.Ez, center=mp.Vector3())])
    s = sim._init_structure()
    assert s.gv.n == [16, 16, 16] and s.gv.io == [-16, -16, -16]
    src = mp.Source(mp.GaussianSource(1.0, fwidth=1.0), mp.Ez, center=mp.Vector3(),
                    size=mp.Vector3(1, 0, 0))  # line sources are in scope
    assert src.size.x == 1
    with pytest.raises(ValueError):
        mp.Source(mp.GaussianSource(1.0, fwidth=1.0), mp.Ez)  # neither center nor volume
    with pytest.raises(NotImplementedError):
        mp.Source(mp.GaussianSource(1.0, fwidth=1.0), mp.Ez, center=mp.Vector3(),
                  amp_func_file="x.h5:amp")


def test_time_sinks_follow_reference_enum():
    """TIME_SINKS (python) and the MNL_SINK_* enum (include/meep_nl_amd.h) list
    meep::time_sink in its order (src/meep.hpp:1610-1633)."""
    import re
    from meep_nl_amd import core
    hdr = open(os.path.join(ROOT, "include", "meep_nl_amd.h")).read()
    body = re.search(r"enum \{\s*(MNL_SINK_CONNECTING.*?)MNL_NUM_TIME_SINKS", hdr, re.S).group(1)
    names = [n.strip() for n in body.split(",") if n.strip()]
    assert len(names) == len(core.TIME_SINKS) == 22
    ref = ["Connecting", "Stepping", "Boundaries", "MpiAllTime", "MpiOneTime", "FieldOutput",
           "FourierTransforming", "MPBTime", "GetFarfieldsTime", "Other", "FieldUpdateB",
           "FieldUpdateH", "FieldUpdateD", "FieldUpdateE", "BoundarySteppingB",
           "BoundarySteppingWH", "BoundarySteppingPH", "BoundarySteppingH", "BoundarySteppingD",
           "BoundarySteppingWE", "BoundarySteppingPE", "BoundarySteppingE"]
    assert [k for k, _ in core.TIME_SINKS] == ref


def test_verbosity_singleton():
    import meep_nl_amd as mp
    v = mp.verbosity
    old = v.get()
    try:
        mp.verbosity(2)
        assert v.meep == 2 and mp.simulation.Verbosity() is v
        v.meep = 0
        assert mp.verbosity() == 0
        mp.quiet(False)
        assert v.get() == 1
    finally:
        v.set(old)
