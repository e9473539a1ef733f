"""Timing and progress reporting (src/time.cpp:130-215 print_times /
output_times / time_spent_on, src/step.cpp:44-56 "on time step", and the
python run loop's "Meep progress" / "run N finished" lines,
python/simulation.py:2795-2855, 5468-5489)."""
import re

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _sim(mp, **kw):
    return mp.Simulation(cell_size=mp.Vector3(6, 5), resolution=20,
                         boundary_layers=[mp.PML(1.0)],
                         sources=[mp.Source(mp.GaussianSource(0.5, fwidth=0.2), mp.Ez,
                                            center=mp.Vector3(0.1, -0.2))], **kw)


def test_print_times_and_output_times(capfd, tmp_path):
    import meep_nl_amd as mp
    from meep_nl_amd import core
    mp.verbosity(1)
    sim = _sim(mp)
    sim.run(until=20)
    out = capfd.readouterr().out
    assert re.search(r"run 0 finished at t = 20(\.0)? \(\d+ timesteps\)", out), out
    sim.run(until=5)
    assert "run 1 finished" in capfd.readouterr().out
    stepping = sim.time_spent_on(1)  # meep::Stepping
    assert len(stepping) == 1 and stepping[0] > 0
    assert sim.mean_time_spent_on(1) == stepping[0]
    data = sim.get_timing_data()
    assert len(data) == len(core.TIME_SINKS) == 22
    # profiling on: the unfused 2-D updates are timed per phase
    assert sum(data[k][0] for k in (10, 11, 12, 13)) > 0
    sim.print_times()
    out = capfd.readouterr().out
    assert "Field time usage:" in out
    assert re.search(r"^ {12}time stepping: [0-9.e+-]+ s$", out, re.M), out
    assert re.search(r"^ {9}updating E field: [0-9.e+-]+ s$", out, re.M), out
    sim.output_times(str(tmp_path / "times"))
    rows = (tmp_path / "times.csv").read_text().splitlines()
    assert rows[0].split(", ") == [label for _, label in core.TIME_SINKS]
    vals = [float(v) for v in rows[1].split(", ")]
    assert len(rows) == 2 and np.isclose(vals[1], stepping[0], rtol=1e-5)
    sim.fields.reset_timers()
    assert sim.time_spent_on(1) == [0.0]


def test_progress_messages(capfd):
    """Meep progress lines every progress_interval seconds of a timed run; the
    native "on time step N (time=T), S s/step" line every 4 s of stepping."""
    import meep_nl_amd as mp
    from meep_nl_amd import core
    mp.verbosity(1)
    sim = _sim(mp, progress_interval=0.2)
    sim.run(until=400)
    out = capfd.readouterr().out
    m = re.findall(r"Meep progress: ([0-9.e+-]+)/400(\.0)? = ([0-9.]+)% done in ([0-9.]+)s, "
                   r"([0-9.]+)s to go", out)
    assert m, out[-2000:]
    assert all(0 < float(x[0]) <= 400 for x in m)
    # native line: 3-D 160^3 stepped for > 4 s of wall time
    gv = core.GridVolume(3, [160, 160, 160], 10.0, [-160, -160, -160])
    f = core.Fields(core.Structure(gv))
    f.add_gaussian_source(2, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, 0.05), 1.0)
    import time
    t0 = time.time()
    while time.time() - t0 < 5.0:
        f.step(500)
    out = capfd.readouterr().out
    lines = re.findall(r"^on time step (\d+) \(time=([0-9.e+-]+)\), ([0-9.e+-]+) s/step$", out, re.M)
    assert lines, out[-2000:]
    n, t, sps = lines[-1]
    assert float(t) == pytest.approx(int(n) * f.dt, rel=1e-5)
    assert 0 < float(sps) < 0.1
    mp.verbosity(0)
    f.step(2000)
    assert "on time step" not in capfd.readouterr().out
    mp.verbosity(1)
