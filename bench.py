#!/usr/bin/env python3
"""Benchmark of the MI355X fields::step() hot path (BASELINE.json metric).

Headline workload (weak scaling): BASELINE configs[2] -- 3-D dielectric
waveguide (eps = 12 core |y|,|z| < 0.5 along x, eps_averaging=False) + PML(1.0)
on all faces, resolution 10, fp64, real fields, Ez Gaussian current source
(GaussianSource(0.15, fwidth=0.1)) at (0.05, 0.05, 0.05).  Each GPU owns a
512^3-cell z-slab: the global grid is 512 x 512 x (512*N), so N=1 is exactly
the 512^3 headline and per-GPU work is fixed as N grows.

A "step" is one fields::step() (src/step.cpp:35-140) over the whole grid.
value = (all cells * K) / max-over-ranks wall time, in Mcells*steps/s.

At N=1 the same JSON line also carries the other single-GPU BASELINE configs,
measured in the same run ("configs"): C2 256^3 vacuum + PML, C4 256^3 Kerr +
Lorentzian slab, and C4's chi(2) Newton-Raphson sub-variant (NR solves/s).

BASELINE configs[4] (C5: 1024x512x512 cells z-slab-decomposed over 8 GPUs) is
--workload c5: vacuum + PML(1.0), 512 x 512 x 128 cells per GPU, global
512 x 512 x (128*N) (the long axis is the slab axis z).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--size S] [--vacuum]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

--gpus N without a launcher starts N ranks under torch.distributed.run (child
processes).  Ranks sharing a GPU (MNL_BENCH_DEVICE, or fewer GPUs than ranks)
exchange ghost planes over the IPC transport, otherwise over RCCL.
Prints ONE JSON line on rank 0 (with "roofline" and "cpu_baseline").
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
WORKLOADS = {
    "waveguide": "C3 3-D dielectric waveguide eps=12 core + PML(1.0)",
    "vacuum": "C3-vacuum 3-D vacuum + PML(1.0)",
    "c2": "C2 3-D vacuum box + PML(1.0), Ez Gaussian at (0.05,0.05,0.05)",
    "kerr": "C4 3-D Kerr chi3 + Lorentzian slab |z|<2 + PML(1.0), Ex source at z=-3 amp 50",
    "kerr_nr": "C4-NR: C4 + chi2 0.5 and chi1inv off-diagonal 1e-3 in the box |x|,|y|<3, "
               "|z|<1.5 (Newton-Raphson E update)",
    "c5": "C5 3-D vacuum + PML(1.0), z-slab decomposed, per GPU S x S x S/4 cells "
          "(S=512: 512x512x128 per GPU, 512x512x1024 = the 1024x512x512 domain at N=8)",
}
NR_BOX = (-3.0, 3.0, -3.0, 3.0, -1.5, 1.5)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-tune", action="store_true",
                    help="keep the default knobs (skip Fields.tune before the warm-up)")
    ap.add_argument("--size", type=int, default=512, help="cells per side of each GPU's slab")
    ap.add_argument("--vacuum", action="store_true", help="north-star vacuum variant (no core)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the C2 / C4 / C4-NR measurements (N=1)")
    ap.add_argument("--extra-size", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--flux", type=int, default=0,
                    help="add N DFT flux planes (x-normal, whole cross-section; decimation 1)")
    ap.add_argument("--nfreq", type=int, default=50, help="frequencies per flux plane")
    ap.add_argument("--no-events", action="store_true",
                    help="diagnostics: no per-kernel HIP events in the timed region")
    ap.add_argument("--no-parity", action="store_true",
                    help="N > 1: skip the C5 self-check against the one-rank fixture")
    ap.add_argument("--no-smi", action="store_true",
                    help="do not query rocm-smi for clocks / power (gpu_state)")
    return ap.parse_args()


def build_fields(workload, size, rank, world, device, nid, zslabs=None):
    """Structure + fields of one workload on this rank (global grid
    size x size x size*world, center_origin, res 10, Courant 0.5; zslabs: the global grid
    of that many slabs whatever the rank count, e.g. the whole C5 grid on one rank)."""
    from meep_nl_amd import core
    import numpy as np
    n = [size, size, (size // 4 if workload == "c5" else size) * (zslabs or world)]
    io = [-(v - (v & 1)) for v in n]  # center_origin()
    gv = core.GridVolume(3, n, 10.0, io)
    s = core.Structure(gv, 0.5)
    s.add_pml(1.0)
    big = 1e9
    if workload in ("kerr", "kerr_nr"):  # |z| < 2: eps 2.25, chi3 1e-2, Lorentzian(1.1, 0.05, 0.5)
        slab = [-big, big, -big, big, -2.0, 2.0]
        s.set_box(0, slab, 2.25)
        s.set_box(2, slab, 1e-2)
        k = s.add_lorentzian(1.1, 0.05, [None, None, None])
        s.set_box(3, slab, 0.5, index=k)
        if workload == "kerr_nr":  # chi2 + off-diagonal chi1inv rows: the NR branch
            x0, x1, y0, y1, z0, z1 = NR_BOX
            s.set_box(1, list(NR_BOX), 0.5)
            for c in range(3):
                x, y, z = gv.coords(c)
                inside = (x > x0) & (x < x1) & (y > y0) & (y < y1) & (z > z0) & (z < z1)
                off = np.where(inside, 1e-3, 0.0)
                del x, y, z, inside
                for d in range(3):
                    if d != c:
                        s.set_chi1inv(c, d, off)
                del off
        f = core.Fields(s, device=device, rank=rank, nranks=world, nccl_id=nid)
        f.add_gaussian_source(0, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, -3.0), 50.0,
                              is_integrated=False)
        return gv, s, f
    if workload == "waveguide":
        s.set_box(0, [-big, big, -0.5 + 1e-12, 0.5 - 1e-12, -0.5 + 1e-12, 0.5 - 1e-12], 12.0)
    f = core.Fields(s, device=device, rank=rank, nranks=world, nccl_id=nid)
    f.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0,
                          is_integrated=False)
    return gv, s, f


def nr_voxels(gv):
    """E points on which the NR branch runs: every E component point inside the
    chi2 / off-diagonal box (non-PML, all three rows present there)."""
    import numpy as np
    x0, x1, y0, y1, z0, z1 = NR_BOX
    lo, hi = (x0, y0, z0), (x1, y1, z1)
    n = 0
    for c in range(3):
        m = 1
        for d in range(3):
            j = np.arange(gv.n[d] + 1)
            ax = (gv.io[d] + 2 * j + gv.shift(c, d)) * (0.5 / gv.a)
            m *= int(np.sum((ax > lo[d]) & (ax < hi[d])))
        n += m
    return n


def roofline(f, kind=0):
    """Roofline object of the dominant kernel: algorithmic bytes per launch over
    its average duration from HIP events on its own stream."""
    n_launch, k_ms, k_bytes = f.kernel_stats(kind)
    avg_ms = k_ms / max(n_launch, 1)
    achieved = k_bytes / (avg_ms * 1e-3) / 1e9 if n_launch and avg_ms > 0 else 0.0
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": (("fused_tile_kernel + fused_general_kernel concurrently on a CU split "
                        "(tile kernel: lean tiles + per-direction PML bodies; general kernel: the "
                        "polarization chunks with the Lorentzian P update); one step, both "
                        "launches' bytes over the span of both"
                        if f.tile_mode() and f.fused_concurrent() else
                        "fused_tile_kernel (one persistent launch over the fused box: lean "
                        "tiles + per-direction PML bodies; curl B + H + curl D + E, one pass)"
                        if f.tile_mode() else
                        "fused_kernel + fused_general_kernel concurrently (whole step, one pass)"
                        if f.kernel_stats(2)[0] == 0 else
                        "fused_kernel (lean tiles: curl B + curl D + E=chi1inv*D, one pass)")
                       if f.fused_active() else "curl_kernel<B, interior> (step_db(B_stuff))"),
            "bytes_per_launch": k_bytes, "avg_launch_ms": round(avg_ms, 4),
            "launches": n_launch}
    tb = f.tb_info() if f.fused_active() else {"active": False}
    t_n, t_ms, t_bytes = f.kernel_stats(5)
    if tb["active"] and t_n:
        # temporal blocking: a pair of steps is three persistent
        # launches (the two-step kernel over L2, then the tile kernel over the rim twice); the
        # algorithmic bytes of a pair are the two-step items' two steps (B, D read once and
        # written once, palette words of mixed items, border points' step n+1) plus two rim
        # steps.  frac_one_step_model prices the same pair at the one-step model (two steps of
        # the tile kernel's bytes), i.e. the HBM rate a one-step kernel would need.
        t_avg = t_ms / t_n
        achieved = t_bytes / (t_avg * 1e-3) / 1e9
        r_n, r_ms, r_bytes = f.kernel_stats(6)
        roof.update({
            "kernel": ("tb2_kernel (two-step z-march over the lean region L2) + 2 x "
                       "fused_tile_kernel over the rim items (PML, walls, ring, source holes; "
                       "x-face strips in the narrow 16 x 63 strip body), one pair of steps"),
            "bytes_per_launch": t_bytes, "avg_launch_ms": round(t_avg, 4), "launches": t_n,
            "launch_unit": "pair of steps (all its launches)",
            "achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
            "steps_per_launch": 2,
            "frac_one_step_model": round(2.0 * k_bytes / (t_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "temporal_blocking": tb})
        if r_n:
            r_avg = r_ms / r_n
            roof["rim_alone"] = {
                "kernel": "fused_tile_kernel over the rim items alone (the last pair's second "
                          "rim step of a batch), included in the pair time above",
                "bytes_per_launch": r_bytes, "avg_launch_ms": round(r_avg, 4), "launches": r_n}
        if n_launch:  # one-step launches of the same run (odd leftovers)
            roof["tile_kernel_one_step"] = {"bytes_per_launch": k_bytes, "launches": n_launch,
                                            "avg_launch_ms": round(avg_ms, 4)}
    if f.fused_active():  # the PML / boundary tiles run in the second fused kernel
        g_n, g_ms, g_bytes = f.kernel_stats(2)
        if g_n:
            g_avg = g_ms / g_n
            roof["general_kernel"] = {
                "kernel": ("fused_general_kernel (polarization chunks, same pass)" if f.tile_mode()
                           else "fused_general_kernel (PML / boundary tiles, same pass)"),
                "bytes_per_launch": g_bytes, "avg_launch_ms": round(g_avg, 4),
                "achieved": round(g_bytes / (g_avg * 1e-3) / 1e9, 1)}
    return roof


def _traffic_file():
    """profiles/pmc_traffic.json and the hash of THIS kernel source, or (None, None)."""
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(tpath):
        return None, None
    try:
        import hashlib
        with open(tpath) as fh:
            tj = json.load(fh)
        with open(os.path.join(ROOT, "meep_nl_amd", "csrc", "mnl_kernels.hip"), "rb") as fh:
            khash = hashlib.sha256(fh.read()).hexdigest()[:16]
        return tj, khash
    except (OSError, ValueError):
        return None, None


def pmc_traffic(size, vacuum):
    """HBM bytes per launch of the headline's dominant kernel (the pair of temporal
    blocking) from the committed PMC profile of THIS kernel source
    (profiles/pmc_traffic.json), else None."""
    tj, khash = _traffic_file()
    try:
        if (tj and tj.get("size") == size and tj.get("vacuum", False) == vacuum
                and tj.get("kernels_hash") == khash):
            return round(tj["hbm_bytes_per_launch"])
    except (KeyError, TypeError):
        return None
    return None


def pmc_traffic_config(workload, size, tb_active):
    """The same for a BASELINE sub-config (configs.<workload>): its entry
    <workload>_<size>_<tb|1s> in pmc_traffic.json "configs" (pairs or one-step stepping,
    profiled with this kernel source), else None."""
    tj, khash = _traffic_file()
    try:
        e = (tj or {}).get("configs", {}).get(f"{workload}_{size}_{'tb' if tb_active else '1s'}")
        if e and e.get("kernels_hash") == khash:
            return round(e["hbm_bytes_per_launch"])
    except (KeyError, TypeError, AttributeError):
        return None
    return None


SMI_CMD = ["rocm-smi", "--showclocks", "--showpower", "--showtemp", "--showmaxpower",
           "--showperflevel", "--json"]


def gpu_state_start():
    """Start a read-only rocm-smi query of clocks, power and temperature in a child
    process (so it can sample while the GPU is stepping), or None."""
    import subprocess
    try:
        return subprocess.Popen(SMI_CMD, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                text=True)
    except OSError:
        return None


def gpu_state_finish(proc):
    """Parse the query started by gpu_state_start: per card, the clock / power /
    temperature / perf-level fields.  Recorded in the bench line so the box-to-box
    spread of one kernel can be attributed to clocks or to page placement (VERDICT r03,
    weak 5).  Never fails the bench."""
    import subprocess
    if proc is None:
        return {"error": "rocm-smi not started"}
    try:
        out_s, err_s = proc.communicate(timeout=30)
        js = json.loads(out_s[out_s.find("{"):]) if "{" in out_s else {}
    except (OSError, ValueError, subprocess.SubprocessError) as e:
        proc.kill()
        return {"error": str(e)[:200]}
    keep = ("sclk", "mclk", "fclk", "socclk", "power", "temp", "perf")
    out = {}
    for card, vals in js.items():
        if isinstance(vals, dict):
            out[card] = {k: v for k, v in vals.items() if any(w in k.lower() for w in keep)}
    return out or {"error": "no rocm-smi data", "rc": proc.returncode, "stderr": err_s[-200:]}


def add_flux_planes(f, gv, planes, nfreq):
    """N x-normal DFT flux planes through the whole cross-section, nfreq frequencies each,
    decimation 1 (fields::add_dft_flux, src/dft.cpp:578-640)."""
    hx = 0.5 * gv.n[0] / 10.0
    hy, hz = 0.5 * gv.n[1] / 10.0, 0.5 * gv.n[2] / 10.0
    freqs = [0.1 + 0.1 * i / max(nfreq - 1, 1) for i in range(nfreq)]
    for i in range(planes):
        x = -hx + 2 * hx * (i + 1) / (planes + 1) + 0.05
        f.add_dft_flux([([x, -hy, -hz], [x, hy, hz], 0, 1.0)], freqs, 1)


def measure_extra(workload, size, steps, warmup, tune=True, flux=0, nfreq=50):
    """One single-GPU BASELINE config in the same process: warm-up, K timed
    steps (stream-synchronized), its own roofline.  flux > 0: that many DFT flux planes
    (add_flux_planes) sampled and accumulated every step inside the timed region."""
    dev = int(os.environ.get("MNL_BENCH_DEVICE", "0"))
    gv, s, f = build_fields(workload, size, 0, 1, dev, None)
    if flux:
        add_flux_planes(f, gv, flux, nfreq)
    zc = f.tune() if tune else None
    f.step(warmup)
    if flux:  # no DFT update of the warm-up left buffered for the timed region
        f.dft_flush()
    f.set_profiling(True)
    t0 = time.perf_counter()
    f.step(steps)
    if flux:  # the accumulation of every timed update inside the timed region
        f.dft_flush()
    el = time.perf_counter() - t0
    cells = float(size) ** 3
    bpc, _ = f.traffic_model()
    out = {"workload": WORKLOADS[workload] + f", {size}^3 cells, res 10, real fields, fp64" +
                       (f", {flux} x-normal DFT flux planes x {nfreq} frequencies (decimation 1)"
                        if flux else ""),
           "value": round(cells * steps / el / 1e6, 1), "unit": "Mcells*steps/s",
           "ms_per_step": round(el / steps * 1e3, 4), "steps": steps, "warmup": warmup,
           "fused": f.fused_active(), "tuned_zchunk_gen_cus": zc, "model_bytes_per_cell_step": round(bpc, 2),
           "model_fraction_of_peak": round(bpc * cells / (el / steps) / 1e9 / HBM_PEAK_GBS, 4),
           "roofline": roofline(f)}
    tb_on = f.fused_active() and f.tb_info()["active"]
    out["roofline"]["traffic"] = (pmc_traffic_config(workload + (f"_flux{flux}" if flux else ""),
                                                     size, tb_on) if f.fused_active() else None)
    if workload == "kerr_nr":
        nv = nr_voxels(gv)
        e_n, e_ms, _ = f.kernel_stats(4)
        out["nr"] = {"metric": "chi(2) Newton-Raphson solves/s", "nr_voxels_per_step": nv,
                     "solves_per_s_whole_step": round(nv * steps / el, 1),
                     "solves_per_s_e_update": round(nv * e_n / (e_ms * 1e-3), 1) if e_ms else None,
                     "e_update_ms_per_step": round(e_ms / max(e_n, 1), 4),
                     "nr_random_fallbacks": f.nr_fallbacks(),
                     "bound": "latency/compute (per-voxel 3x3 Newton iterations), not HBM"}
    if flux:  # the DFT updates (sampling + accumulation) of every timed step
        d_n, d_ms, d_bytes = f.kernel_stats(3)
        out["dft"] = {"planes": flux, "nfreq": nfreq, "updates": d_n,
                      "ms_per_step": round(d_ms / max(steps, 1), 4),
                      "bytes_per_update": d_bytes}
        out["temporal_blocking"] = bool(f.fused_active() and f.tb_info()["active"])
    if f.fused_active():  # per-step time of each launch family: which one dominates
        parts = {}
        for name, kind in (("fused_tile_kernel", 0),
                           ("fused_general_kernel (polarization chunks)", 2),
                           ("E phase (kerr_nr: NR box update_e_kernel<NR> + nr_hard + "
                            "update_pols)", 4)):
            n, ms, _ = f.kernel_stats(kind)
            if n:
                parts[name] = round(ms / n, 4)
        if parts:
            out["step_breakdown_ms"] = parts
            out["roofline"]["dominant_kernel"] = max(parts, key=parts.get)
    del f, s
    gc.collect()
    return out


def rank_breakdown(f, rank, el_ms_per_step):
    """Per-rank timing of a multi-rank run (HIP events): per pair of steps the two-step
    kernel, the rim launches (R1 + both parts of R2), the slab-face chains on the comm stream
    (top plane's step, sources, B/H and E plane exchanges: two per pair, beside the main
    stream) and the main stream's waits for a chain's E ghost (two per pair); one-step steps
    (odd leftovers) are not in it."""
    pairs, pair_ms, _ = f.kernel_stats(5)
    _, rim_ms, _ = f.kernel_stats(6)
    _, chain_ms, _ = f.kernel_stats(7)
    _, wait_ms, _ = f.kernel_stats(8)
    n = max(pairs, 1)
    return {"rank": rank, "pairs": pairs, "ms_per_step": round(el_ms_per_step, 4),
            "pair_ms": round(pair_ms / n, 4), "two_step_ms": round((pair_ms - rim_ms) / n, 4),
            "rim_ms": round(rim_ms / n, 4), "face_chain_ms": round(chain_ms / n, 4),
            "exchange_wait_ms": round(wait_ms / n, 4)}


C5_STEPS = 7  # 1 step (unfused after initialize_field) + 3 pairs of steps


def c5_fixture_path(n):
    return os.path.join(ROOT, "tests", "golden", f"c5_parity_{n[0]}x{n[1]}x{n[2]}.npz")


def plane_checksums(arr):
    """Per plane of the last (z, the slab) axis: the sum over the plane of each value's IEEE
    bit pattern times an odd weight of its (x, y, z) position, mod 2^64 (the same function as
    tests/scenarios.plane_checksums).  Entries a rank does not own are 0 in its get_array and
    every entry has one owner, so the ranks' checksums add up (mod 2^64) to the one-rank
    run's exactly when every entry is bitwise equal."""
    import numpy as np
    a = np.ascontiguousarray(arr).view(np.uint64)
    nx, ny, nz = a.shape
    out = np.zeros(nz, dtype=np.uint64)
    ky = (np.arange(ny, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))[:, None]
    kz = (np.arange(nz, dtype=np.uint64) * np.uint64(0xD6E8FEB86659FD93))[None, :]
    with np.errstate(over="ignore"):
        for i in range(nx):
            w = (np.uint64(i) * np.uint64(0xBF58476D1CE4E5B9) + ky + kz) | np.uint64(1)
            out += (a[i] * w).sum(axis=0, dtype=np.uint64)
    return out


def c5_parity_run(size, zslabs, rank, world, device, nid, log=None):
    """The C5 self-check state on this rank: the C5 grid of zslabs slabs (S x S x S/4 each),
    seeded random D and B everywhere (tests/scenarios.sc_c5_full's seeds), stepped 1 + 6
    (an unfused first step, then three pairs: the slab-face chains, both rim launches and the
    two-step kernel all carry data); returns the grid, this rank's per-plane checksums of all
    twelve components [12, nz] and the run's facts."""
    import numpy as np
    gv, s, f = build_fields("c5", size, rank, world, device, nid, zslabs=zslabs)
    for c in (6, 7, 8, 9, 10, 11):
        v = np.random.default_rng(7 + 31 * c).standard_normal(gv.shape())
        f.initialize_field(c, v)
        del v
        if log:
            log(f"initialized component {c}")
    f.step(1)
    f.step(C5_STEPS - 1)
    cs = np.stack([plane_checksums(f.get_array(c)) for c in range(12)])
    facts = {"t": f.t, "transport": f.transport(), "ranks": world,
             "temporal_blocking": bool(f.fused_active() and f.tb_info()["active"])}
    del f, s
    gc.collect()
    return gv, cs, facts


def c5_parity_compare(parts, ref):
    """Sum the ranks' plane checksums (mod 2^64) and compare with the one-rank fixture:
    (equal, [(component, plane), ...] of the first differing planes)."""
    import numpy as np
    with np.errstate(over="ignore"):
        tot = np.zeros_like(ref)
        for p in parts:
            tot = tot + p.astype(np.uint64)
    bad = np.argwhere(tot != ref)
    return bad.size == 0, [tuple(int(x) for x in b) for b in bad[:8]]


def c5_parity(args, rank, world, device, dist):
    """Self-validation of a multi-rank run: step the C5 grid of this run
    from seeded random fields over the ranks (RCCL with one GPU per rank) and compare every
    plane of every component, summed over the ranks, with the one-rank fixture
    tests/golden/c5_parity_<grid>.npz (tools/make_c5_fixture.py) -- the reference's chunk
    invariance (tests/three_d.cpp:35-39) at 0.  None when no fixture covers this grid."""
    import numpy as np
    from meep_nl_amd import core
    n = [args.size, args.size, args.size // 4 * world]
    path = c5_fixture_path(n)
    have = os.path.exists(path)
    if not have:
        return {"c5_parity": None, "reason": f"no fixture for the {n[0]}x{n[1]}x{n[2]} grid"}
    transport, _ = core.pick_transport(world, int(os.environ.get("LOCAL_RANK", "0")))
    obj = [core.comm_id(world, transport) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    t0 = time.perf_counter()
    gv, cs, facts = c5_parity_run(args.size, world, rank, world, device, obj[0])
    parts = [None] * world
    dist.all_gather_object(parts, cs)
    out = {"grid": n, "steps": C5_STEPS, "ranks": world, "transport": facts["transport"],
           "temporal_blocking": facts["temporal_blocking"], "fixture": os.path.relpath(path, ROOT)}
    if rank == 0:
        with np.load(path, allow_pickle=False) as z:
            ref = z["checksums"]
        ok, bad = c5_parity_compare(parts, ref)
        out.update({"c5_parity": bool(ok), "bad_planes": bad})
    out["seconds"] = round(time.perf_counter() - t0, 1)
    return out


def measure_c5(args, rank, world, device, dist):
    """BASELINE C5 on the ranks of this run: per GPU a S x S x S/4 z-slab of the vacuum +
    PML(1.0) grid (S = --size; 512: the 1024x512x512 domain at N = 8), tuned, warmed up,
    K steps between barriers, max over ranks."""
    from meep_nl_amd import core
    import torch
    transport, _ = core.pick_transport(world, int(os.environ.get("LOCAL_RANK", "0")))
    obj = [core.comm_id(world, transport) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    gv, s, f = build_fields("c5", args.size, rank, world, device, obj[0])
    zc = None if args.no_tune else f.tune()
    f.step(args.warmup)
    dist.barrier()
    f.set_profiling(not args.no_events)
    t0 = time.perf_counter()
    f.step(args.steps)
    dist.barrier()
    el_own = time.perf_counter() - t0
    t = torch.tensor([el_own], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    per_rank = [None] * world
    dist.all_gather_object(per_rank, rank_breakdown(f, rank, el_own / args.steps * 1e3))
    cells = float(gv.n[0]) * gv.n[1] * gv.n[2]
    out = {"workload": WORKLOADS["c5"] + f", global {gv.n[0]}x{gv.n[1]}x{gv.n[2]} cells "
                       f"({world} z-slabs), res 10, real fields",
           "value": round(cells * args.steps / el / 1e6, 1), "unit": "Mcells*steps/s",
           "ms_per_step": round(el / args.steps * 1e3, 4), "steps": args.steps,
           "n_gpus": world, "scaling": "weak", "transport": f.transport(),
           "fused": f.fused_active(), "tuned_zchunk_gen_cus": zc,
           "temporal_blocking": f.fused_active() and f.tb_info()["active"],
           "per_rank": per_rank}
    del f, s
    gc.collect()
    return out


def cpu_baseline(args):
    """Time the oracle (CPU restatement, oracle/) on the headline config itself: the
    512^3 waveguide (eps = 12 core) + PML(1.0) with the same Gaussian source, OpenMP on this
    host's share of cores (OMP_NUM_THREADS; 16 per GPU on the driver's boxes), a few steps
    after two untimed ones (about 10-20 s of stepping at ~1 s per step)."""
    from oracle import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    orc.set_threads(threads)
    import numpy as np
    L = args.size
    t_setup = time.perf_counter()
    o = orc.Oracle(3, [L, L, L], 10.0, 0.5, [-L, -L, -L])
    o.add_pml(1.0)
    if not args.vacuum:
        for c in (0, 1, 2):
            x, y, z = o.coords(c)
            del x
            core = (np.abs(y) < 0.5 - 1e-12) & (np.abs(z) < 0.5 - 1e-12)
            del y, z
            o.set_chi1inv(c, c, np.where(core, 1 / 12.0, 1.0))
            del core
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    t_setup = time.perf_counter() - t_setup
    o.step(2)
    steps, t0 = 0, time.perf_counter()
    while True:
        o.step(2)
        steps += 2
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or steps >= 400:
            break
    v = L ** 3 * steps / el / 1e6
    wl = "vacuum" if args.vacuum else "waveguide (eps = 12 core)"
    return {"value": round(v, 2), "unit": "Mcells*steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ CPU restatement of the headline config itself: {L}^3 {wl} + "
                      f"PML(1.0), Ez Gaussian source, {steps} timed steps after 2 untimed in "
                      f"{el:.1f} s (set-up {t_setup:.0f} s not timed), OpenMP {threads} threads "
                      f"(OMP_NUM_THREADS; the host reports {os.cpu_count()} CPUs)"}


def launch_ranks(args):
    """--gpus N > 1 without a launcher: start N ranks under torch.distributed.run
    as CHILD processes (this process never touches the GPU) and exit with their
    status."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.workload in ("vacuum", "c5"):
        args.vacuum = True
    if args.workload is None:
        args.workload = "vacuum" if args.vacuum else "waveguide"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}\n")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    nid = None
    device = local_rank
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # the gloo group (host-side barriers, the max over ranks) prints its connection
        # messages to stdout from C++: send them to stderr, stdout carries the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        from meep_nl_amd import core
        transport, device = core.pick_transport(world, local_rank)
        obj = [core.comm_id(world, transport) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nid = obj[0]
    elif os.environ.get("MNL_BENCH_DEVICE"):
        device = int(os.environ["MNL_BENCH_DEVICE"])
    from meep_nl_amd import core as _core
    _core.set_verbosity(0)  # no "on time step" lines: stdout carries the one JSON line
    try:
        gv, s, f = build_fields(args.workload, args.size, rank, world, device, nid)
    except RuntimeError as e:  # a failed RCCL setup names RCCL and exits non-zero
        sys.stderr.write(f"bench.py rank {rank}: {e}\n")
        sys.exit(3)
    if args.flux:  # on-device DFT flux monitors
        add_flux_planes(f, gv, args.flux, args.nfreq)

    def barrier():
        if dist is not None:
            dist.barrier()

    # untimed set-up: the fused step's knobs timed over real steps (identical results)
    zc = None if args.no_tune else f.tune()
    f.step(args.warmup)
    # GPU clocks / power sampled while this rank keeps stepping (untimed, <= 10 s), and
    # again right after the timed region
    state_busy = None
    if not args.no_smi:
        proc = gpu_state_start() if rank == 0 else None
        if world == 1:
            t_s = time.perf_counter()
            while proc is not None and proc.poll() is None and time.perf_counter() - t_s < 10:
                f.step(10)
        else:  # every rank steps the same count (the steps are collective)
            f.step(100)
        if proc is not None:
            state_busy = gpu_state_finish(proc)
    if args.flux:  # no DFT update of the warm-up left buffered for the timed region
        f.dft_flush()
    barrier()
    f.set_profiling(not args.no_events)
    t0 = time.perf_counter()
    f.step(args.steps)  # returns after the device work is complete (stream synchronized)
    if args.flux:  # the accumulation of every timed update inside the timed region
        f.dft_flush()
    barrier()
    el = time.perf_counter() - t0
    el_own = el
    state_after = gpu_state_finish(gpu_state_start()) if rank == 0 and not args.no_smi else None
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    bpc, _ = f.traffic_model()
    total_cells = float(gv.n[0]) * gv.n[1] * gv.n[2]
    value = total_cells * args.steps / el / 1e6
    roof = roofline(f)
    roof["traffic"] = (pmc_traffic(args.size, args.vacuum)
                       if f.fused_active() and args.workload in ("waveguide", "vacuum") else None)
    if world > 1 and os.environ.get("MNL_BENCH_DEVICE"):
        roof["note"] = ("all ranks share one GPU (rehearsal): the per-launch rate is a share "
                        "of one device, not a roofline fraction")
    if args.flux:
        d_n, d_ms, d_bytes = f.kernel_stats(3)
        if d_n:
            d_avg = d_ms / d_n
            roof["dft"] = {"kernel": f"dft_update_kernel x{args.flux} planes, {args.nfreq} freqs",
                           "bytes_per_step": d_bytes, "avg_step_ms": round(d_avg, 4),
                           "achieved": round(d_bytes / (d_avg * 1e-3) / 1e9, 1)}
    transport = f.transport()
    fused = f.fused_active()
    per_rank = None
    if dist is not None:  # per-rank pair / rim / slab-face chain / exchange-wait breakdown
        per_rank = [None] * world
        dist.all_gather_object(per_rank, rank_breakdown(f, rank, el_own / args.steps * 1e3))
    del f, s
    gc.collect()
    extra = None
    if world > 1 and not args.no_extra and args.workload != "c5":
        # BASELINE configs[4] (C5) in the same multi-GPU run: 512 x 512 x 128 vacuum + PML
        # per GPU, its own communicator, timed the same way (max over ranks)
        try:
            extra = {"c5": measure_c5(args, rank, world, device, dist)}
        except Exception as e:  # never hides the headline number
            extra = {"c5": {"error": str(e)}}
    parity = None
    if world > 1 and not args.no_parity:
        try:
            parity = c5_parity(args, rank, world, device, dist)
        except Exception as e:  # never hides the headline number
            parity = {"c5_parity": False, "error": str(e)}
    if rank != 0:
        if dist is not None:
            dist.barrier()
        return
    if world == 1 and not args.no_extra and not args.flux:
        extra = {}
        for wl in ("c2", "kerr", "kerr_nr"):
            try:
                extra[wl] = measure_extra(wl, args.extra_size, 20, 5, not args.no_tune)
            except Exception as e:  # an extra config must never hide the headline number
                extra[wl] = {"error": str(e)}
        # the headline grid with 4 whole-cross-section flux planes x 50 frequencies (SURVEY.md
        # 8(f) row 1 on the C3 config; the same monitors as --flux 4); 64 timed steps = two
        # whole accumulation blocks (32 updates per pass over the DFT arrays), all of them
        # accumulated inside the timed region
        try:
            extra["flux4"] = measure_extra(args.workload, args.size, 64, 6, not args.no_tune,
                                           flux=4, nfreq=50)
        except Exception as e:
            extra["flux4"] = {"error": str(e)}
    cpu = None
    if world == 1 and not args.no_cpu and args.workload in ("waveguide", "vacuum") and not args.flux:
        try:
            cpu = cpu_baseline(args)
        except Exception as e:  # the baseline must never hide the GPU number
            cpu = {"error": str(e)}
    out = {
        "metric": "Mcells*steps/s (Yee cells x timesteps / s)",
        "value": round(value, 1),
        "unit": "Mcells*steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Gaussian point source; fields start at zero)",
        "config": {
            "workload": WORKLOADS[args.workload] +
                        (f", {args.size}x{args.size}x({args.size // 4}*N) cells" if args.workload == "c5"
                         else f", {args.size}x{args.size}x({args.size}*N) cells") +
                        ", res 10, real fields" +
                        (", Ez Gaussian current at (0.05,0.05,0.05)"
                         if args.workload in ("waveguide", "vacuum", "c5") else ""),
            "grid": list(gv.n), "per_gpu_cells": int(gv.n[0]) * int(gv.n[1]) * int(gv.n[2]) // world,
            "parallelism": f"z-slab x{world}",
            "transport": transport, "fused": fused, "tuned_zchunk_gen_cus": zc,
            "flux_planes": args.flux, "flux_nfreq": args.nfreq if args.flux else 0,
            "model_bytes_per_cell_step": bpc,
            "model_fraction_of_peak": round(bpc * total_cells / world / (el / args.steps) / 1e9
                                            / HBM_PEAK_GBS, 4)},
        "roofline": roof,
        "per_rank": per_rank,
        "cpu_baseline": cpu,
        "configs": extra,
        "c5_parity": parity.get("c5_parity") if parity else None,
        "c5_parity_ranks": world if parity else None,
        "c5_parity_check": parity,
        "gpu_state": {"while_stepping": state_busy, "after": state_after},
    }
    print(json.dumps(out))
    sys.stdout.flush()
    if dist is not None:
        dist.barrier()


if __name__ == "__main__":
    main()
