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


def test_traffic_lookup_is_hash_and_mode_gated(tmp_path, monkeypatch):
    """roofline.traffic comes from profiles/pmc_traffic.json only for the kernel source it
    was measured on, the same size, and (sub-configs) the same stepping mode."""
    import hashlib
    import json
    import bench
    (tmp_path / "profiles").mkdir()
    (tmp_path / "meep_nl_amd" / "csrc").mkdir(parents=True)
    src = tmp_path / "meep_nl_amd" / "csrc" / "mnl_kernels.hip"
    src.write_text("// kernels v1\n")
    h = hashlib.sha256(src.read_bytes()).hexdigest()[:16]
    doc = {"kernels_hash": h, "size": 512, "vacuum": False, "hbm_bytes_per_launch": 26.9e9,
           "configs": {"c2_256_1s": {"kernels_hash": h, "hbm_bytes_per_launch": 2.38e9},
                       "kerr_256_1s": {"kernels_hash": "stale", "hbm_bytes_per_launch": 2.0e9}}}
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(doc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic(512, False) == round(26.9e9)
    assert bench.pmc_traffic(256, False) is None
    assert bench.pmc_traffic(512, True) is None
    assert bench.pmc_traffic_config("c2", 256, False) == round(2.38e9)
    assert bench.pmc_traffic_config("c2", 256, True) is None       # measured one-step only
    assert bench.pmc_traffic_config("kerr", 256, False) is None    # other kernel source
    src.write_text("// kernels v2\n")                              # the kernels changed
    assert bench.pmc_traffic(512, False) is None
    assert bench.pmc_traffic_config("c2", 256, False) is None
