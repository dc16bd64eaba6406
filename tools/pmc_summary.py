"""Summarise rocprofv3 --pmc counter CSVs: per-dispatch mean of each counter for kernels
whose name contains a filter string, plus per-wave cycle breakdowns."""
import collections
import csv
import glob
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else ""
for d in sorted(glob.glob(sys.argv[1] + "/*/run_counter_collection.csv")):
    agg, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(d)):
        if pat and pat not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    m = {k: v / max(n[k], 1) for k, v in agg.items()}
    out = {k: f"{v:.4g}" for k, v in m.items()}
    if "SQ_WAVES" in m:
        w = m["SQ_WAVES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in m:
                out[k + "/wave(cyc)"] = f"{4 * m[k] / w:.4g}"
    print(d.split("/")[-2], out)
