"""One rank of a multi-process run (tests/test_gpu_mp.py): the slab
decomposition through mnl_fields_create_dist in separate processes, as the
multi-GPU path runs it (one process per slab), with the transport named by the
128-byte id (IPC when the ranks share one GPU).

  python tests/mp_worker.py RANK NRANKS ID_HEX[,ID_HEX...] OUT_DIR CASE [CASE ...]

(one communicator id per case)

Writes OUT_DIR/<case>.rank<R>.npz: every component array (this rank's owned
entries, zeros elsewhere) plus the collective results the case asks for
(get_field, fluxes, array slices -- identical on every rank)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import scenarios as S  # noqa: E402


def make_dist(rank, nranks, nid):
    class DistSim(S.ProductSim):
        def _fields(self):
            if self.f is None:
                dev = int(os.environ.get("MNL_MP_DEVICE", "0"))
                self.f = self.core.Fields(self.s, device=dev, rank=rank, nranks=nranks,
                                          nccl_id=nid)
            return self.f
    return DistSim


def run_case(name, make):
    extra = {}
    if name == "c5_full":  # full-size C5: per-plane checksums, not arrays (2 GB each)
        def log(m):
            print(f"c5_full: {m}", flush=True)
        o = S.sc_c5_full(make, log=log)
        log("stepped")
        cs = np.stack([S.plane_checksums(o.get_array(c)) for c in range(12)])
        return {"cs": cs, "transport": np.array(o._fields().transport()),
                "tb": np.array([o._fields().tb_info()["active"]]), "t": np.array([o.t])}
    if name == "vacuum_pml":
        o = S.sc_vacuum_pml_3d(make)
    elif name == "big_box":
        o = S.sc_big_box_3d(make, steps=16)
    elif name == "big_box_tuned":  # z-chunk tuner on every rank (collective steps), then 30
        o = S.sc_big_box_3d(make, steps=0)
        extra["zchunk"] = np.array([o._fields().tune(reps=1)[0]])
        o.step(30 - o.t)
    elif name == "kerr_lorentz":
        o = S.sc_kerr_lorentz_3d(make)
    elif name == "nr_dispersive":
        o = S.sc_nr_pml_dispersive(make)
    elif name == "nr_seam":
        o = S.sc_nr_isrc_seam(make)
    elif name == "averaged_up":
        o = S.sc_averaged(make, upstream=True)
    elif name == "c5_small":
        o = S.sc_c5_small(make)
    elif name.startswith("fuzz"):  # a seeded random configuration (tests/test_gpu_fuzz.py)
        from test_gpu_fuzz import build
        o, _ = build(make, int(name[4:]))
    elif name == "flux":
        o, hs = S.sc_flux_3d(make, steps=40)
        for k, h in enumerate(hs):
            extra[f"flux{k}"] = o.flux(h)
        # slices bigger than the 64-value allreduce staging buffer (growth path)
        extra["slice_plane"] = o.get_array_slice(2, [-1.6, -1.6, 0.3], [1.6, 1.6, 0.3])
        extra["slice_box"] = o.get_array_slice(4, [-0.7, -0.5, -1.2], [0.9, 0.6, 1.1])
        extra["point"] = np.array([o.get_field(2, (0.11, -0.23, 0.37))])
    else:
        raise SystemExit(f"unknown case {name}")
    arrs = {f"c{c}": o.get_array(c) for c in range(12)}
    arrs.update(extra)
    arrs["transport"] = np.array(o._fields().transport())
    arrs["tb"] = np.array([o._fields().tb_info()["active"]])  # pairs of steps
    arrs["t"] = np.array([o.t])
    return arrs


def main():
    rank, nranks = int(sys.argv[1]), int(sys.argv[2])
    ids = [bytes.fromhex(h) for h in sys.argv[3].split(",")]
    out = sys.argv[4]
    names = sys.argv[5:]
    assert len(ids) == len(names)
    for nid, name in zip(ids, names):
        res = run_case(name, make_dist(rank, nranks, nid))
        np.savez(os.path.join(out, f"{name}.rank{rank}.npz"), **res)
        print(f"rank {rank}: {name} done", flush=True)


if __name__ == "__main__":
    main()
