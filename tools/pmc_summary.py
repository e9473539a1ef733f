#!/usr/bin/env python3
"""Summarise rocprofv3 stats / PMC runs (tools/gpu.sh prof: and pmc: steps, or the round-1
to-3 layout gpurun_out/prof_<tag>/{stats,fetch,write}) into profiles/.

Per kernel: calls, average duration (kernel-trace stats pass), HBM bytes per
launch from the PMC passes, corrected as MI355X_MICROARCH.md prescribes and
as calibrated on this pool with tools/micro/fetch_calib.hip (profiles/
r01_fetch_calibration.json): FETCH_SIZE (KiB) reports exactly half of the
bytes read for 4-, 8- and 16-byte-per-lane loads -> bytes = 2 * 1024 * FETCH_SIZE;
WRITE_SIZE (KiB) is exact -> bytes = 1024 * WRITE_SIZE.

  python tools/pmc_summary.py gpurun_out/prof_r01 profiles/r01_pmc_512wg.json \
      [--traffic profiles/pmc_traffic.json --size 512 --kernel fused_kernel]

--traffic also writes the file bench.py reads for roofline.traffic, keyed by the
hash of meep_nl_amd/csrc/mnl_kernels.hip so a stale profile is never reported
for a changed kernel.
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels_hash():
    with open(os.path.join(ROOT, "meep_nl_amd", "csrc", "mnl_kernels.hip"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("mnl::", "")


def counters(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def write_headline(path, doc):
    """the headline entry of the traffic file; the sub-config entries ("configs") are kept"""
    try:
        with open(path) as fh:
            old = json.load(fh)
    except (OSError, ValueError):
        old = {}
    if "configs" in old:
        doc["configs"] = old["configs"]
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--traffic")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--vacuum", action="store_true")
    ap.add_argument("--kernel", default="fused_kernel")
    ap.add_argument("--pair", action="store_true",
                    help="temporal blocking: the traffic of a pair of steps = tb2_kernel + 2 x "
                         "fused_tile_kernel (the rim launches)")
    ap.add_argument("--config", metavar="WORKLOAD",
                    help="with --traffic: write the entry configs.<WORKLOAD>_<size>_<tb|1s> of the file "
                         "(a bench.py sub-config; --kernel names its dominant kernel, --pair a "
                         "temporal-blocking pair) and keep the rest of the file")
    ap.add_argument("--dirs", nargs=3, metavar=("STATS", "FETCH", "WRITE"),
                    help="separate directories of the stats / FETCH_SIZE / WRITE_SIZE runs "
                         "(tools/gpu.sh prof: / pmc: steps) instead of src/{stats,fetch,write}")
    a = ap.parse_args()
    sub = dict(zip(("stats", "fetch", "write"), a.dirs)) if a.dirs else {
        k: os.path.join(a.src, k) for k in ("stats", "fetch", "write")}
    res = {}
    for f in glob.glob(os.path.join(sub["stats"], "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            res.setdefault(k, {})
            res[k]["calls"] = int(r["Calls"])
            res[k]["avg_ms"] = float(r["AverageNs"]) / 1e6
    fe, wr = counters(sub["fetch"]), counters(sub["write"])
    sq, tcc = counters(os.path.join(a.src, "sq")), counters(os.path.join(a.src, "tcc"))
    sq2 = counters(os.path.join(a.src, "sq2"))
    for k in set(fe) | set(wr):
        e = res.setdefault(k, {})
        if fe[k]["FETCH_SIZE"]:
            e["read_bytes"] = 2 * 1024 * sum(fe[k]["FETCH_SIZE"]) / len(fe[k]["FETCH_SIZE"])
        if wr[k]["WRITE_SIZE"]:
            e["write_bytes"] = 1024 * sum(wr[k]["WRITE_SIZE"]) / len(wr[k]["WRITE_SIZE"])
        if "read_bytes" in e and "write_bytes" in e:
            e["hbm_bytes"] = e["read_bytes"] + e["write_bytes"]
            if e.get("avg_ms"):
                e["hbm_GBps"] = e["hbm_bytes"] / (e["avg_ms"] * 1e-3) / 1e9
        for src in (sq, tcc, sq2):
            for c, v in src.get(k, {}).items():
                e[c] = sum(v) / len(v)
    doc = {"source": a.src, "kernels_hash": kernels_hash(),
           "corrections": "read = 2*1024*FETCH_SIZE, write = 1024*WRITE_SIZE (calibrated)",
           "kernels": res}
    with open(a.dst, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    print(json.dumps({k: {kk: (round(vv, 4) if isinstance(vv, float) else vv)
                          for kk, vv in v.items() if kk in ("avg_ms", "hbm_bytes", "hbm_GBps")}
                      for k, v in res.items()}, indent=1))
    if a.traffic and a.config:
        try:
            with open(a.traffic) as fh:
                doc_t = json.load(fh)
        except (OSError, ValueError):
            doc_t = {}
        if a.pair:
            tb = [k for k in res if k.startswith("tb2_kernel") and "hbm_bytes" in res[k]]
            rim = [k for k in res if k.startswith("fused_tile_kernel") and "hbm_bytes" in res[k]]
            if not (tb and rim):
                return
            entry = {"kernel": "pair: tb2_kernel + 2 x fused_tile_kernel (rim)", "tb": True,
                     "hbm_bytes_per_launch": res[tb[0]]["hbm_bytes"] + 2 * res[rim[0]]["hbm_bytes"]}
        else:
            # --kernel a,b: kernels launched once per step side by side (the tile kernel and the
            # polarization chunks' general kernel on a CU split): their bytes add up
            ks = []
            for pre in a.kernel.split(","):
                m = [k for k in res if k.startswith(pre) and "hbm_bytes" in res[k]]
                if not m:
                    return
                ks.append(m[0])
            entry = {"kernel": " + ".join(ks), "tb": False,
                     "hbm_bytes_per_launch": sum(res[k]["hbm_bytes"] for k in ks),
                     "per_kernel": {k: res[k]["hbm_bytes"] for k in ks}}
        entry.update({"kernels_hash": kernels_hash(), "profile": os.path.basename(a.dst)})
        doc_t.setdefault("configs", {})[f"{a.config}_{a.size}_{'tb' if a.pair else '1s'}"] = entry
        with open(a.traffic, "w") as fh:
            json.dump(doc_t, fh, indent=1)
        return
    if a.traffic and a.pair:
        tb = [k for k in res if k.startswith("tb2_kernel") and "hbm_bytes" in res[k]]
        rim = [k for k in res if k.startswith("fused_tile_kernel") and "hbm_bytes" in res[k]]
        if tb and rim:
            hb = res[tb[0]]["hbm_bytes"] + 2 * res[rim[0]]["hbm_bytes"]
            doc_t = {"kernels_hash": kernels_hash(), "size": a.size, "vacuum": a.vacuum,
                     "kernel": "pair: tb2_kernel + 2 x fused_tile_kernel (rim)",
                     "unit": "pair of steps", "hbm_bytes_per_launch": hb,
                     "tb2_bytes": res[tb[0]]["hbm_bytes"],
                     "rim_bytes": res[rim[0]]["hbm_bytes"],
                     "profile": os.path.basename(a.dst)}
            write_headline(a.traffic, doc_t)
        return
    if a.traffic:
        ks = [k for k in res if k.startswith(a.kernel) and "hbm_bytes" in res[k]]
        if ks:
            k = ks[0]
            write_headline(a.traffic, {"kernels_hash": kernels_hash(), "size": a.size,
                                       "vacuum": a.vacuum, "kernel": k,
                                       "hbm_bytes_per_launch": res[k]["hbm_bytes"],
                                       "profile": os.path.basename(a.dst)})


if __name__ == "__main__":
    main()
