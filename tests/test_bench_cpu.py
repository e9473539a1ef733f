"""bench.py's driver contract on the CPU side (no GPU): the default command is the
single-GPU headline run with a warm-up, the knobs the driver passes parse, and the
workload names cover BASELINE.json's configs."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_defaults_and_driver_flags(monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.steps, a.warmup, a.size) == (1, 60, 10, 512)
    assert not a.no_tune and a.workload is None
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "7", "--warmup", "3",
                                      "--no-tune", "--workload", "c5"])
    a = bench.parse()
    assert (a.gpus, a.steps, a.warmup, a.no_tune, a.workload) == (8, 7, 3, True, "c5")


def test_workloads_cover_the_baseline_configs():
    import bench
    # configs[1] C2, configs[2] C3 (waveguide; vacuum = the north star's variant),
    # configs[3] C4 (kerr; kerr_nr its chi(2) sub-variant), configs[4] C5
    assert {"c2", "waveguide", "vacuum", "kerr", "kerr_nr", "c5"} <= set(bench.WORKLOADS)


def test_help_runs_without_a_gpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "--no-tune" in r.stdout
