"""Multi-process slabs: the distributed path (mnl_fields_create_dist, the
three-stream fused step, the chunk-0 side stream, collective get_field / flux /
array slices) with one process per slab, as torch.distributed.run launches it
on a multi-GPU node.  On the one-GPU test box the ranks share the device, so the
transport is IPC (RCCL refuses two ranks on one GPU: "Duplicate GPU detected");
every other line of the multi-rank code is the one the RCCL run executes.

Parity: the sum of the ranks' owned entries equals the CPU oracle bit for bit
(the reference's chunk invariance, tests/three_d.cpp:35-39, at 0 instead of
1e-9); fluxes to rel 1e-12 (per-rank partial sums), slices and get_field
bitwise, identical on every rank."""
import os
import subprocess
import sys

import numpy as np
import pytest

from scenarios import make_oracle
import scenarios as S

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

HERE = os.path.dirname(os.path.abspath(__file__))
CASES2 = ["vacuum_pml", "big_box", "big_box_tuned", "kerr_lorentz", "nr_dispersive", "nr_seam",
          "flux", "fuzz0", "fuzz2", "fuzz9", "fuzz16"]
CASES3 = ["big_box", "flux", "averaged_up", "fuzz5", "fuzz24"]
CASES8 = ["c5_small"]  # BASELINE C5's decomposition (8 z-slabs) at reduced x-y


def _launch(nranks, cases, out, stream=False, timeout=400):
    """One worker process per rank; stream=True: their output goes straight to this
    process's real stderr (progress of long cases), else it is collected for failures."""
    from meep_nl_amd import core
    ids = ",".join(core.ipc_id(nranks).hex() for _ in cases)
    env = dict(os.environ, MNL_IPC_TIMEOUT="120")
    pipe = None if stream else subprocess.PIPE
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mp_worker.py"), str(r),
                               str(nranks), ids, str(out)] + cases, env=env,
                              stdout=pipe if pipe else sys.__stderr__,
                              stderr=subprocess.STDOUT, text=True)
             for r in range(nranks)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o or "")
    for p, o in zip(procs, logs):
        assert p.returncode == 0, o[-3000:]


@pytest.fixture(scope="module")
def mp_runs(tmp_path_factory):
    out = {}
    for n, cases in ((2, CASES2), (3, CASES3), (8, CASES8)):
        d = tmp_path_factory.mktemp(f"mp{n}")
        _launch(n, cases, d)
        out[n] = d
    return out


def _load(d, name, nranks):
    return [dict(np.load(os.path.join(d, f"{name}.rank{r}.npz"))) for r in range(nranks)]


def _oracle(name):
    if name == "vacuum_pml":
        return S.sc_vacuum_pml_3d(make_oracle), {}
    if name == "big_box":
        return S.sc_big_box_3d(make_oracle, steps=16), {}
    if name == "big_box_tuned":
        return S.sc_big_box_3d(make_oracle, steps=30), {}
    if name == "kerr_lorentz":
        return S.sc_kerr_lorentz_3d(make_oracle), {}
    if name == "nr_dispersive":
        return S.sc_nr_pml_dispersive(make_oracle), {}
    if name == "nr_seam":
        return S.sc_nr_isrc_seam(make_oracle), {}
    if name == "averaged_up":
        return S.sc_averaged(make_oracle, upstream=True), {}
    if name == "c5_small":
        return S.sc_c5_small(make_oracle), {}
    if name.startswith("fuzz"):
        from test_gpu_fuzz import build
        return build(make_oracle, int(name[4:]))[0], {}
    o, hs = S.sc_flux_3d(make_oracle, steps=40)
    ex = {f"flux{k}": o.flux(h) for k, h in enumerate(hs)}
    ex["slice_plane"] = o.get_array_slice(2, [-1.6, -1.6, 0.3], [1.6, 1.6, 0.3])
    ex["slice_box"] = o.get_array_slice(4, [-0.7, -0.5, -1.2], [0.9, 0.6, 1.1])
    ex["point"] = np.array([o.get_field(2, (0.11, -0.23, 0.37))])
    return o, ex


@pytest.mark.parametrize("nranks,name", [(2, c) for c in CASES2] + [(3, c) for c in CASES3] +
                         [(8, c) for c in CASES8])
def test_multiprocess_slabs_bitwise(mp_runs, nranks, name):
    ranks = _load(mp_runs[nranks], name, nranks)
    assert all(str(r["transport"]) == "ipc" for r in ranks)
    o, ex = _oracle(name)
    for c in range(12):
        got = sum(r[f"c{c}"] for r in ranks)
        ref = o.get_array(c)
        assert got.shape == ref.shape
        d = float(np.max(np.abs(got - ref))) if ref.size else 0.0
        assert d == 0.0, (c, d)
    if name == "big_box_tuned":  # every rank tuned (the same choice: max over ranks), then 30
        assert all(int(r["zchunk"][0]) in (0, 16, 20, 24, 32, 48) for r in ranks)
        assert len({int(r["zchunk"][0]) for r in ranks}) == 1
    if name in ("big_box", "big_box_tuned", "c5_small"):  # multi-rank temporal blocking
        assert all(bool(r["tb"][0]) for r in ranks)
    for k, v in ex.items():
        for r in ranks:  # collectives: every rank holds the same result
            np.testing.assert_array_equal(r[k], ranks[0][k])
        if k.startswith("flux"):
            np.testing.assert_allclose(ranks[0][k], v, rtol=1e-12, atol=1e-300)
        else:
            np.testing.assert_array_equal(ranks[0][k], v)
    assert int(ranks[0]["t"][0]) == o.t


def test_rccl_selftest():
    """The RCCL wrappers the slab exchange uses (grouped ncclSend/ncclRecv on a
    stream, ncclAllReduce with the growable staging buffer) on a one-rank
    communicator: send-to-self and allreduce return the data intact."""
    from meep_nl_amd import core
    core.rccl_selftest(0, 1 << 20)
    core.rccl_selftest(0, 37)


def test_c5_full_size_chunk_invariance(tmp_path):
    """BASELINE configs[4] (C5) at full size: 8 processes stepping 512 x 512 x 128 z-slabs of
    the 512 x 512 x 1024 vacuum + PML grid (IPC transport: the ranks share this GPU) against one
    rank stepping the whole grid, from the same random fields, 1 + 6 steps (three pairs of
    multi-rank temporal blocking).  The reference's chunk invariance (tests/three_d.cpp:35-39)
    at 0: every entry of all twelve components bitwise equal, checked through per-plane
    position-weighted bit-pattern sums (scenarios.plane_checksums), whose rank sums equal the
    one-rank sums exactly when the arrays do."""
    _launch(8, ["c5_full"], tmp_path, stream=True, timeout=900)
    ranks = _load(tmp_path, "c5_full", 8)
    assert all(str(r["transport"]) == "ipc" for r in ranks)
    assert all(bool(r["tb"][0]) for r in ranks)  # the slabs stepped pairs
    with np.errstate(over="ignore"):
        got = sum(r["cs"] for r in ranks[1:]) + ranks[0]["cs"]
    def log(m):
        sys.__stderr__.write(f"c5_full one rank: {m}\n")
        sys.__stderr__.flush()
    o = S.sc_c5_full(S.ProductSim, log=log)
    assert o._fields().tb_info()["active"]
    assert int(ranks[0]["t"][0]) == o.t
    for c in range(12):
        ref = S.plane_checksums(o.get_array(c))
        bad = np.nonzero(got[c] != ref)[0]
        assert bad.size == 0, (c, bad[:10].tolist())
    log("all planes equal")


def test_bench_two_ranks_self_check():
    """bench.py --gpus 2 as the driver runs it (torch.distributed.run children; here both ranks
    share this GPU over IPC): the line carries the multi-GPU self-check -- the C5 grid of the
    run stepped from seeded random fields over both ranks, every plane of every component
    summed over the ranks equal to the one-rank fixture tests/golden/c5_parity_256x256x128.npz
    (tools/make_c5_fixture.py) -- as c5_parity true with the rank count."""
    import json
    root = os.path.dirname(HERE)
    env = dict(os.environ, MNL_BENCH_DEVICE="0", MNL_IPC_TIMEOUT="300")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--size",
                        "256", "--steps", "4", "--warmup", "2", "--no-tune", "--no-smi"],
                       env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    chk = line["c5_parity_check"]
    assert line["c5_parity"] is True and line["c5_parity_ranks"] == 2, chk
    assert chk["transport"] == "ipc" and chk["temporal_blocking"] and chk["bad_planes"] == []
    assert chk["grid"] == [256, 256, 128] and chk["steps"] == 7
