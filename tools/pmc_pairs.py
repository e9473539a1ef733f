#!/usr/bin/env python3
"""Per-pair summary of a temporal-blocking run (round 6): rocprofv3 kernel-trace / stats pass and
separate FETCH_SIZE / WRITE_SIZE passes of the same bench.py command (tools/gpu.sh prof: / pmc:
steps).  Since round 6 a pair of steps is the two-step kernel, the first rim launch in two parts
(its non-strip items beside the two-step kernel on a side stream, the narrow strips after it)
and the second rim launch, so per-launch averages of fused_tile_kernel no longer equal "one rim
step": this groups the dispatches by pair (every fused_tile_kernel dispatch from one tb2_kernel
dispatch to the next) and reports per pair

  * tb2 / rim / pair HBM bytes (read = 2 * 1024 * FETCH_SIZE, write = 1024 * WRITE_SIZE, as
    calibrated in profiles/r01_fetch_calibration.json and MI355X_MICROARCH.md "HBM"),
  * the pair's span in the trace (start of tb2_kernel to the end of the pair's last rim
    dispatch) and the kernels' own durations,

medians over the pairs (the first pair after a plan change is dropped).  With --traffic the
headline entry of profiles/pmc_traffic.json (or, with --config W, its entry configs.W_<size>_tb)
is written, keyed by the hash of meep_nl_amd/csrc/mnl_kernels.hip.

  python tools/pmc_pairs.py STATS FETCH WRITE OUT.json [--traffic profiles/pmc_traffic.json
         --size 512 [--config c2]]
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels_hash():
    with open(os.path.join(ROOT, "meep_nl_amd", "csrc", "mnl_kernels.hip"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def kind(name):
    if "tb2_kernel" in name:
        return "tb2"
    if "fused_tile_kernel" in name or "fused_general_kernel" in name:  # rim / polarization
        return "tile"
    return None


def merge(a, b):
    """two tb2_kernel dispatches of one pair (the interior items on their own stream, then the
    others): bytes add up, the span is their union"""
    m = dict(a)
    if "bytes" in a:
        m["bytes"] = a["bytes"] + b["bytes"]
    if "start" in a:
        m["start"], m["end"] = min(a["start"], b["start"]), max(a["end"], b["end"])
        m["busy"] = a.get("busy", a["end"] - a["start"]) + (b["end"] - b["start"])
    return m


def per_pair(disp):
    """dispatch list [(id, kind, value...)] in dispatch order -> list of (tb2, [tile, ...]);
    consecutive tb2_kernel dispatches belong to one pair"""
    pairs, cur = [], None
    for d in disp:
        if d["kind"] == "tb2":
            if cur and not cur["tile"]:
                cur["tb2"] = merge(cur["tb2"], d)
                continue
            if cur:
                pairs.append(cur)
            cur = {"tb2": d, "tile": []}
        elif d["kind"] == "tile" and cur:
            cur["tile"].append(d)
    if cur:
        pairs.append(cur)
    return pairs


def counter_pairs(d, counter, scale):
    disp = []
    for r in rows(d, "*counter_collection.csv"):
        k = kind(r["Kernel_Name"])
        if k and r["Counter_Name"] == counter:
            disp.append({"id": int(r["Dispatch_Id"]), "kind": k,
                         "bytes": float(r["Counter_Value"]) * scale})
    disp.sort(key=lambda x: x["id"])
    return per_pair(disp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--traffic")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--config")
    ap.add_argument("--vacuum", action="store_true")
    a = ap.parse_args()
    # trace: spans and durations per pair
    tr = []
    for r in rows(a.stats, "*kernel_trace.csv"):
        k = kind(r["Kernel_Name"])
        if k:
            tr.append({"id": int(r["Dispatch_Id"]), "kind": k, "start": int(r["Start_Timestamp"]),
                       "end": int(r["End_Timestamp"])})
    tr.sort(key=lambda x: x["id"])
    tpairs = [p for p in per_pair(tr) if len(p["tile"]) >= 2][1:]
    span = [(max([p["tb2"]["end"]] + [t["end"] for t in p["tile"]]) - p["tb2"]["start"]) / 1e6
            for p in tpairs]
    tb2_ms = [p["tb2"].get("busy", p["tb2"]["end"] - p["tb2"]["start"]) / 1e6 for p in tpairs]
    last_rim_ms = [(p["tile"][-1]["end"] - p["tile"][-1]["start"]) / 1e6 for p in tpairs]
    rd = [p for p in counter_pairs(a.fetch, "FETCH_SIZE", 2048.0) if len(p["tile"]) >= 2][1:]
    wr = [p for p in counter_pairs(a.write, "WRITE_SIZE", 1024.0) if len(p["tile"]) >= 2][1:]
    med = statistics.median

    def side(pp):
        return (med([p["tb2"]["bytes"] for p in pp]),
                med([sum(t["bytes"] for t in p["tile"]) for p in pp]),
                med([len(p["tile"]) for p in pp]))
    tb_r, rim_r, nl = side(rd)
    tb_w, rim_w, _ = side(wr)
    doc = {"kernels_hash": kernels_hash(), "pairs": len(tpairs),
           "rim_dispatches_per_pair": nl,
           "corrections": "read = 2*1024*FETCH_SIZE, write = 1024*WRITE_SIZE (calibrated)",
           "tb2_bytes": tb_r + tb_w, "tb2_read_bytes": tb_r, "tb2_write_bytes": tb_w,
           "rim_bytes_per_pair": rim_r + rim_w, "rim_read_bytes_per_pair": rim_r,
           "rim_write_bytes_per_pair": rim_w,
           "pair_bytes": tb_r + tb_w + rim_r + rim_w,
           "pair_span_ms": med(span) if span else None, "tb2_ms": med(tb2_ms) if tb2_ms else None,
           "last_rim_launch_ms": med(last_rim_ms) if last_rim_ms else None,
           "source": [a.stats, a.fetch, a.write]}
    if doc["pair_span_ms"]:
        doc["pair_GBps_memory_side"] = doc["pair_bytes"] / (doc["pair_span_ms"] * 1e-3) / 1e9
    if doc["tb2_ms"]:
        doc["tb2_GBps_memory_side"] = doc["tb2_bytes"] / (doc["tb2_ms"] * 1e-3) / 1e9
    with open(a.out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in doc.items()
                      if k != "source"}, indent=1))
    if not a.traffic:
        return
    try:
        with open(a.traffic) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        t = {}
    entry = {"kernels_hash": kernels_hash(), "size": a.size, "vacuum": a.vacuum,
             "kernel": "pair: tb2_kernel + the fused_tile_kernel rim dispatches of the pair",
             "unit": "pair of steps", "tb": True, "hbm_bytes_per_launch": doc["pair_bytes"],
             "tb2_bytes": doc["tb2_bytes"], "rim_bytes_per_pair": doc["rim_bytes_per_pair"],
             "profile": os.path.relpath(a.out, ROOT)}
    if a.config:
        t.setdefault("configs", {})[f"{a.config}_{a.size}_tb"] = entry
    else:
        keep = t.get("configs")
        t = entry
        if keep:
            t["configs"] = keep
    with open(a.traffic, "w") as fh:
        json.dump(t, fh, indent=1)


if __name__ == "__main__":
    main()
