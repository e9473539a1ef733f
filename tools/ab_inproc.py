"""In-process A/B of a scheduling option of the fused step (Fields.set_schedule: identical
results, different scheduling): one process, one allocation, the two settings alternated
--rounds times (--values: two or more settings, rotated), --steps timed steps each after a
re-plan warm-up, medians reported.  Between
processes the same kernel varies with page placement, so options are
compared inside one process.

  python tools/ab_inproc.py --option narrow [--workload waveguide] [--size 512] [--rounds 4]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--option", required=True, choices=["narrow", "dft_pal", "res", "res_tb2", "res_rim", "dft_cmp", "rim_zchunk", "nr_early", "tb_zchunk", "tb_ox", "tb_px", "tb_pol", "r1_beside", "tb_lint", "r2_lpt", "strip_zchunk", "src_guard", "events"])
    ap.add_argument("--workload", default="waveguide")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--retune", action="store_true",
                    help="tune again after every switch (options that change the tuner's choice)")
    ap.add_argument("--values", default="0,1",
                    help="the two settings compared (integers; 0,1 = off / on)")
    ap.add_argument("--flux", type=int, default=0,
                    help="N x-normal DFT flux planes as in bench.py --flux")
    ap.add_argument("--nfreq", type=int, default=50)
    ap.add_argument("--fresh", action="store_true",
                    help="new fields for every measurement (workloads whose cost grows with the "
                         "fields, e.g. kerr_nr's Newton-Raphson fallbacks)")
    ap.add_argument("--json")
    a = ap.parse_args()
    import bench
    from meep_nl_amd import core
    core.set_verbosity(0)
    def build():
        gv, s, f = bench.build_fields(a.workload, a.size, 0, 1, 0, None)
        if a.flux:  # the same monitors as bench.py --flux
            hx, hy, hz = 0.5 * gv.n[0] / 10.0, 0.5 * gv.n[1] / 10.0, 0.5 * gv.n[2] / 10.0
            freqs = [0.1 + 0.1 * i / max(a.nfreq - 1, 1) for i in range(a.nfreq)]
            for i in range(a.flux):
                x = -hx + 2 * hx * (i + 1) / (a.flux + 1) + 0.05
                f.add_dft_flux([([x, -hy, -hz], [x, hy, hz], 0, 1.0)], freqs, 1)
        if a.tune:
            f.tune()
        f.step(6)
        return s, f

    s, f = build()
    vals = [int(x) for x in a.values.split(",")]
    res = {v: [] for v in vals}
    for r in range(a.rounds):
        # rotate every second round and reverse odd rounds, so that each setting runs first
        # in half of the rounds (two values: 0,1 / 1,0 / 1,0 / 0,1 ...; ADVICE r05: the old
        # rotation-then-reverse always ran the first value first with two values)
        k = (r // 2) % len(vals)
        order = vals[k:] + vals[:k]
        for v in (order if r % 2 == 0 else order[::-1]):
            if a.fresh:
                del f, s
                s, f = build()
            if a.option == "events":  # per-launch HIP timing events on / off (bench.py's)
                f.set_profiling(bool(v))
            else:
                f.set_schedule(a.option, v)
            if a.retune:
                f.tune()
            f.step(4)  # re-plan / re-enter the fused mode outside the timed steps
            t0 = time.perf_counter()
            f.step(a.steps)
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            res[v].append(ms)
            print(f"round {r} {a.option}={v}: {ms:.4f} ms/step", flush=True)
    out = {"option": a.option, "workload": a.workload, "size": a.size, "steps": a.steps,
           "flux_planes": a.flux, "nfreq": a.nfreq if a.flux else 0,
           "ms_per_step": {str(k): v for k, v in res.items()},
           "median": {str(k): statistics.median(v) for k, v in res.items()}}
    base = out["median"][str(vals[0])]
    out["gain"] = {str(v): 1.0 - out["median"][str(v)] / base for v in vals[1:]}
    if vals == [0, 1]:
        out["gain"] = out["gain"]["1"]
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
