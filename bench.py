#!/usr/bin/env python3
"""Benchmark of the MI355X fields::step() hot path (BASELINE.json metric).

Workload (weak scaling): BASELINE configs[2] -- 3-D dielectric waveguide
(eps = 12 core |y|,|z| < 0.5 along x, eps_averaging=False) + PML(1.0) on all
faces, resolution 10, fp64, real fields, Ez Gaussian current source
(GaussianSource(0.15, fwidth=0.1)) at (0.05, 0.05, 0.05).  Each GPU owns a
512^3-cell z-slab: the global grid is 512 x 512 x (512*N), so N=1 is exactly
the 512^3 headline and per-GPU work is fixed as N grows.

A "step" is one fields::step() (src/step.cpp:35-140) over the whole grid.
value = (all cells * K) / max-over-ranks wall time, in Mcells*steps/s.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--size S] [--vacuum]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line on rank 0 (with "roofline" and "cpu_baseline").
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=512, help="cells per side of each GPU's slab")
    ap.add_argument("--vacuum", action="store_true", help="north-star vacuum variant (no core)")
    ap.add_argument("--workload", choices=["waveguide", "vacuum", "kerr"], default=None,
                    help="kerr: BASELINE configs[3] (chi3 + Lorentzian slab, unfused path)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--flux", type=int, default=0,
                    help="add N DFT flux planes (x-normal, whole cross-section; decimation 1)")
    ap.add_argument("--nfreq", type=int, default=50, help="frequencies per flux plane")
    ap.add_argument("--no-events", action="store_true",
                    help="diagnostics: no per-kernel HIP events in the timed region")
    return ap.parse_args()


def build_fields(args, rank, world, local_rank, nid):
    from meep_nl_amd import core
    res = 10.0
    n = [args.size, args.size, args.size * world]
    io = [-(v - (v & 1)) for v in n]  # center_origin()
    gv = core.GridVolume(3, n, res, io)
    s = core.Structure(gv, 0.5)
    s.add_pml(1.0)
    if args.workload == "kerr":  # |z| < 2: eps 2.25, chi3 1e-2, Lorentzian(1.1, 0.05, 0.5)
        big = 1e9
        slab = [-big, big, -big, big, -2.0, 2.0]
        s.set_box(0, slab, 2.25)
        s.set_box(2, slab, 1e-2)
        k = s.add_lorentzian(1.1, 0.05, [None, None, None])
        s.set_box(3, slab, 0.5, index=k)
        f = core.Fields(s, device=local_rank, rank=rank, nranks=world, nccl_id=nid)
        f.add_gaussian_source(0, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, -3.0), 50.0,
                              is_integrated=False)
        return gv, s, f
    if not args.vacuum:
        big = 1e9
        s.set_box(0, [-big, big, -0.5 + 1e-12, 0.5 - 1e-12, -0.5 + 1e-12, 0.5 - 1e-12], 12.0)
    f = core.Fields(s, device=local_rank, rank=rank, nranks=world, nccl_id=nid)
    f.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0,
                          is_integrated=False)
    return gv, s, f


def cpu_baseline(args):
    """Time the oracle (CPU restatement, oracle/) on a bounded sample of the same
    workload on this host's cores."""
    from oracle import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    orc.set_threads(threads)
    import numpy as np
    L = 128
    o = orc.Oracle(3, [L, L, L], 10.0, 0.5, [-L, -L, -L])
    o.add_pml(1.0)
    if not args.vacuum:
        for c in (0, 1, 2):
            x, y, z = o.coords(c)
            o.set_chi1inv(c, c, np.where((np.abs(y) < 0.5) & (np.abs(z) < 0.5), 1 / 12.0, 1.0))
    o.add_gaussian_source(2, 0.15, 10.0, 0.0, 100.0, (0.05, 0.05, 0.05), 1.0)
    o.step(2)
    steps, t0 = 0, time.perf_counter()
    while True:
        o.step(2)
        steps += 2
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or steps >= 400:
            break
    v = L ** 3 * steps / el / 1e6
    return {"value": round(v, 2), "unit": "Mcells*steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ CPU restatement, {L}^3 {'vacuum' if args.vacuum else 'waveguide'}"
                      f"+PML(1.0), {steps} steps in {el:.1f} s, OpenMP {threads} threads"}


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
    if args.workload == "vacuum":
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
    transport, device = "single", local_rank
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from meep_nl_amd import core
        transport, device = core.pick_transport(world, local_rank)
        obj = [core.comm_id(world, transport) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nid = obj[0]
    elif os.environ.get("MNL_BENCH_DEVICE"):
        device = int(os.environ["MNL_BENCH_DEVICE"])
    gv, s, f = build_fields(args, rank, world, device, nid)
    if args.flux:  # on-device DFT flux monitors
        hx = 0.5 * gv.n[0] / 10.0
        hy, hz = 0.5 * gv.n[1] / 10.0, 0.5 * gv.n[2] / 10.0
        freqs = [0.1 + 0.1 * i / max(args.nfreq - 1, 1) for i in range(args.nfreq)]
        for i in range(args.flux):
            x = -hx + 2 * hx * (i + 1) / (args.flux + 1) + 0.05
            f.add_dft_flux([([x, -hy, -hz], [x, hy, hz], 0, 1.0)], freqs, 1)

    def barrier():
        if dist is not None:
            dist.barrier()

    f.step(args.warmup)
    barrier()
    f.set_profiling(not args.no_events)
    t0 = time.perf_counter()
    f.step(args.steps)  # returns after the device work is complete (stream synchronized)
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    n_launch, k_ms, k_bytes = f.kernel_stats(0)
    bpc, cells_local = f.traffic_model()
    total_cells = float(gv.n[0]) * gv.n[1] * gv.n[2]
    value = total_cells * args.steps / el / 1e6
    if rank != 0:
        if dist is not None:
            dist.barrier()
        return
    avg_ms = k_ms / max(n_launch, 1)
    achieved = k_bytes / (avg_ms * 1e-3) / 1e9 if n_launch else 0.0
    traffic = None  # HBM bytes per launch from the committed PMC profile of THIS kernel source
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            import hashlib
            with open(tpath) as fh:
                tj = json.load(fh)
            with open(os.path.join(ROOT, "meep_nl_amd", "csrc", "mnl_kernels.hip"), "rb") as fh:
                khash = hashlib.sha256(fh.read()).hexdigest()[:16]
            if (tj.get("size") == args.size and tj.get("vacuum", False) == args.vacuum
                    and tj.get("kernels_hash") == khash):
                traffic = round(tj["hbm_bytes_per_launch"])
        except (OSError, ValueError, KeyError):
            traffic = None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": (("fused_kernel + fused_general_kernel concurrently (whole step, one pass)"
                        if f.kernel_stats(2)[0] == 0 else
                        "fused_kernel (lean tiles: curl B + curl D + E=chi1inv*D, one pass)")
                       if f.fused_active() else "curl_kernel<B, interior> (step_db(B_stuff))"),
            "bytes_per_launch": k_bytes, "avg_launch_ms": round(avg_ms, 4),
            "launches": n_launch}
    if f.fused_active():  # the PML / boundary tiles run in the second fused kernel
        g_n, g_ms, g_bytes = f.kernel_stats(2)
        if g_n:
            g_avg = g_ms / g_n
            roof["general_kernel"] = {
                "kernel": "fused_general_kernel (PML / boundary tiles, same pass)",
                "bytes_per_launch": g_bytes, "avg_launch_ms": round(g_avg, 4),
                "achieved": round(g_bytes / (g_avg * 1e-3) / 1e9, 1)}
    if args.flux:
        d_n, d_ms, d_bytes = f.kernel_stats(3)
        if d_n:
            d_avg = d_ms / d_n
            roof["dft"] = {"kernel": f"dft_update_kernel x{args.flux} planes, {args.nfreq} freqs",
                           "bytes_per_step": d_bytes, "avg_step_ms": round(d_avg, 4),
                           "achieved": round(d_bytes / (d_avg * 1e-3) / 1e9, 1)}
    cpu = None
    if world == 1 and not args.no_cpu and args.workload != "kerr" and not args.flux:
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
            "workload": {"waveguide": "C3 3-D dielectric waveguide eps=12 core + PML(1.0)",
                         "vacuum": "C3-vacuum 3-D vacuum + PML(1.0)",
                         "kerr": "C4 3-D Kerr chi3 + Lorentzian slab |z|<2 + PML(1.0), "
                                 "Ex source at z=-3"}[args.workload] +
                        f", {args.size}x{args.size}x({args.size}*N) cells, res 10, real fields" +
                        (", Ez Gaussian current at (0.05,0.05,0.05)"
                         if args.workload != "kerr" else ""),
            "grid": list(gv.n), "per_gpu_cells": args.size ** 3, "parallelism": f"z-slab x{world}",
            "transport": f.transport(),
            "flux_planes": args.flux, "flux_nfreq": args.nfreq if args.flux else 0,
            "model_bytes_per_cell_step": bpc},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out))
    sys.stdout.flush()
    if dist is not None:
        dist.barrier()


if __name__ == "__main__":
    main()
