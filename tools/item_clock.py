"""Per-item timing of the persistent kernels (diagnostics): steps a
bench workload with MNL_ITEM_CLOCK set, so every item of the tile kernel (one-step launches
and temporal-blocking rim launches) and of the two-step kernel records its start / end wall
clock (100 MHz) and CU, then summarises per launch kind and item body: items, own cells,
workgroup time, ns per cell, and the launches' makespan against the summed item time (the
share of the CUs' time spent in items; the rest is tail / queue / launch overhead).

  python tools/item_clock.py [--workload waveguide] [--size 512] [--steps 8] [--no-tb]
                             [--tune] [--json out.json]
"""
import argparse
import collections
import gc
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MAGIC = 0x4b4c434d4e4d
KIND = {0: "tile (one-step)", 1: "rim (tile kernel, pairs)", 2: "two-step"}
BODY = {0: "lean", 1: "x-PML", 2: "y-PML", 3: "z-PML", 4: "identity", 5: "xyz-PML", 6: "xy-PML",
        7: "xz-PML"}


def read(path):
    raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    recs, i = [], 0
    while i < len(raw):
        assert int(raw[i, 0]) == MAGIC, "bad record stream"
        n = int(raw[i, 2])
        recs.append(raw[i + 1:i + 1 + n])
        i += 1 + n
    return np.concatenate(recs) if recs else np.zeros((0, 8), np.uint64)


def span(v):
    return (v & 0xFFFF, (v >> 16) & 0xFFFF)


def summarise(r):
    t0, t1 = r[:, 0].astype(np.int64), r[:, 1].astype(np.int64)
    kind = (r[:, 2] & 0xFF).astype(int)
    cu = (r[:, 2] >> 8).astype(np.int64)  # persistent workgroup (one per CU)
    code = r[:, 3].astype(np.int64)
    out = {}
    for k in sorted(set(kind.tolist())):
        m = kind == k
        # launches: items of one kind, split where no item of the kind runs for > 20 us
        order = np.argsort(t0[m])
        s0, s1 = t0[m][order], t1[m][order]
        run_end = np.maximum.accumulate(s1)
        cut = np.nonzero(s0[1:] > run_end[:-1] + 2000)[0] + 1
        starts = np.concatenate(([0], cut))
        ends = np.concatenate((cut, [len(s0)]))
        makespan = sum(int(run_end[e - 1] - s0[b]) for b, e in zip(starts, ends)) * 10.0  # ns
        busy = float(np.sum(t1[m] - t0[m])) * 10.0
        ncu = len(set(cu[m].tolist()))
        groups = collections.defaultdict(lambda: [0, 0.0, 0.0])
        for i in np.nonzero(m)[0]:
            if k == 2:
                label = "two-step" + (" (uniform palette)" if code[i] & 64 else "")
                x0, x1 = span(int(r[i, 4]))
                y0, y1 = span(int(r[i, 5]))
                z0, z1 = span(int(r[i, 6]))
                cells = (x1 - x0 + 1) * (y1 - y0 + 1) * (z1 - z0) * 2  # two steps
            else:
                body = (int(code[i]) >> 24) & 7
                x0, x1 = span(int(r[i, 4]))
                y0, y1 = span(int(r[i, 5]))
                z0, z1 = span(int(r[i, 6]))
                w = x1 - x0 + 1
                g3 = int(np.int64(r[i, 7]))
                if g3 >= 0:
                    a, b = span(g3)
                    w += b - a + 1
                cells = w * (y1 - y0 + 1) * (z1 - z0)
                label = f"{BODY[body]} w{min(w, 64):02d} r{y1 - y0 + 1:02d} p{min(z1 - z0, 99):02d}"
            g = groups[label]
            g[0] += 1
            g[1] += cells
            g[2] += float(t1[i] - t0[i]) * 10.0
        rows = sorted(groups.items(), key=lambda kv: -kv[1][2])
        out[KIND.get(k, str(k))] = {
            "launches": len(starts), "items": int(m.sum()), "cus": ncu,
            "makespan_us": round(makespan / 1e3, 1), "item_time_us": round(busy / 1e3, 1),
            "busy_share": round(busy / max(makespan * ncu, 1.0), 3),
            "groups": [{"label": lab, "items": v[0], "cells": v[1], "wg_us": round(v[2] / 1e3, 1),
                        "ns_per_cell": round(v[2] / max(v[1], 1), 4),
                        "us_per_item": round(v[2] / 1e3 / v[0], 2)} for lab, v in rows]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="waveguide")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--no-tb", action="store_true")
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--json")
    ap.add_argument("--top", type=int, default=14)
    a = ap.parse_args()
    fd, path = tempfile.mkstemp(prefix="mnl_clk_", suffix=".bin")
    os.close(fd)
    os.environ["MNL_ITEM_CLOCK"] = path
    if a.no_tb:
        os.environ["MNL_TB"] = "0"
    import bench
    gv, s, f = bench.build_fields(a.workload, a.size, 0, 1, 0, None)
    print("fields built", flush=True)
    if a.tune:
        f.tune()
        print("tuned", flush=True)
    f.step(4)
    print("warm", flush=True)
    open(path, "wb").close()  # keep only the measured steps
    f.step(a.steps)
    print("stepped", flush=True)
    del f, s
    gc.collect()
    res = summarise(read(path))
    os.unlink(path)
    res["config"] = {"workload": a.workload, "size": a.size, "steps": a.steps,
                     "temporal_blocking": not a.no_tb, "tuned": a.tune}
    for k, v in res.items():
        if k == "config":
            continue
        print(f"== {k}: {v['launches']} launches, {v['items']} items on {v['cus']} CUs, makespan "
              f"{v['makespan_us']} us, item time {v['item_time_us']} us, busy {v['busy_share']}")
        for g in v["groups"][:a.top]:
            print(f"   {g['label']:<34s} items {g['items']:6d} cells {g['cells']:12.0f} "
                  f"wg {g['wg_us']:10.1f} us  {g['ns_per_cell']:.4f} ns/cell  "
                  f"{g['us_per_item']:8.2f} us/item")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
