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


def test_c5_parity_check_fires_on_a_corrupted_plane():
    """The multi-GPU self-check (bench.c5_parity): the ranks' plane checksums summed mod 2^64
    equal the one-rank checksums when every entry is bitwise equal, and the check names the
    plane when one value is corrupted, two values are swapped within a plane, or a rank writes
    a plane one position off.  Arrays split over 4 z-slabs, zeros where a rank owns nothing
    (as get_array returns them on a rank)."""
    import numpy as np
    import bench
    from scenarios import plane_checksums as scen_cs
    rng = np.random.default_rng(5)
    nx, ny, nz, nr = 6, 5, 16, 4
    arrs = [rng.standard_normal((nx, ny, nz)) for _ in range(12)]
    ref = np.stack([bench.plane_checksums(a) for a in arrs])
    for a, r in zip(arrs, ref):  # the same function as the tests' scenarios
        assert np.array_equal(scen_cs(a), r)

    def parts(mut=None):
        out = []
        for r in range(nr):
            z0, z1 = nz * r // nr, nz * (r + 1) // nr
            cs = []
            for c, a in enumerate(arrs):
                own = np.zeros_like(a)
                own[:, :, z0:z1] = a[:, :, z0:z1]
                if mut:
                    mut(r, c, own)
                cs.append(bench.plane_checksums(own))
            out.append(np.stack(cs))
        return out

    assert bench.c5_parity_compare(parts(), ref) == (True, [])

    def flip(r, c, own):  # one bit of one value on rank 2, component 7, plane 9
        if (r, c) == (2, 7):
            v = own.view(np.uint64)
            v[3, 1, 9] ^= np.uint64(1)

    ok, bad = bench.c5_parity_compare(parts(flip), ref)
    assert not ok and bad == [(7, 9)]

    def swap(r, c, own):  # two values of one plane exchanged
        if (r, c) == (1, 0):
            own[0, 0, 5], own[1, 2, 5] = own[1, 2, 5].copy(), own[0, 0, 5].copy()

    ok, bad = bench.c5_parity_compare(parts(swap), ref)
    assert not ok and bad == [(0, 5)]

    def shift(r, c, own):  # rank 3 writes its first plane one plane low
        if (r, c) == (3, 11):
            own[:, :, 11] = own[:, :, 12]
            own[:, :, 12] = 0

    ok, bad = bench.c5_parity_compare(parts(shift), ref)
    assert not ok and (11, 11) in bad and (11, 12) in bad


def test_c5_parity_fixtures_are_well_formed():
    """tests/golden/c5_parity_<grid>.npz (tools/make_c5_fixture.py, one-rank GPU runs): one
    uint64 checksum per plane and component of the grid it names, after bench.C5_STEPS steps,
    loadable without pickles.  The driver's multi-GPU grids (512 x 512 x 128N, N = 2, 4, 8)
    are covered."""
    import glob
    import numpy as np
    import bench
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "c5_parity_*.npz")))
    names = {os.path.basename(p) for p in files}
    for nz in (256, 512, 1024):
        assert f"c5_parity_512x512x{nz}.npz" in names
    for p in files:
        with np.load(p, allow_pickle=False) as z:
            cs, grid = z["checksums"], [int(v) for v in z["grid"]]
            assert cs.dtype == np.uint64 and cs.shape == (12, grid[2] + 1)  # n + 1 Yee planes
            assert int(z["steps"][0]) == bench.C5_STEPS == int(z["t"][0])
            assert bench.c5_fixture_path(grid) == p
