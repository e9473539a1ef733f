#!/usr/bin/env python3
"""Per-kernel corrected HBM bytes per launch of tools/pmc_ab.sh variants."""
import collections, csv, glob, os, sys
for d in sorted(glob.glob("gpurun_out/pmcab_*_FETCH_SIZE")):
    i = os.path.basename(d).split("_")[1]
    out = collections.defaultdict(dict)
    for c, scale in (("FETCH_SIZE", 2048), ("WRITE_SIZE", 1024)):
        for f in glob.glob(f"gpurun_out/pmcab_{i}_{c}/**/*counter_collection.csv", recursive=True):
            acc = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mnl::", "")
                acc[k].append(float(r["Counter_Value"]) * scale)
            for k, v in acc.items():
                out[k][c] = sum(v) / len(v)
    for k, v in sorted(out.items()):
        if "fused" in k or "dft" in k:
            print(i, k, {c: round(x / 1e9, 3) for c, x in v.items()}, "GB")
