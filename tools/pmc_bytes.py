"""Per-kernel DRAM traffic from a tools/pmc_hbm_bytes.sh run: for every (kernel, grid)
group the mean per dispatch of each counter, DRAM read bytes (32-byte sectors x 32) and
write bytes (64-byte requests x 64 + the rest x 32)."""
import collections
import csv
import glob
import json
import sys

for d in sorted(glob.glob(sys.argv[1] + "/*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(d)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[(name[:60], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, grid), cs in sorted(agg.items()):
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        rd = m.get("TCC_EA0_RDREQ_DRAM_32B_sum", 0.0) * 32
        wr64 = m.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        wr = wr64 * 64 + (m.get("TCC_EA0_WRREQ_sum", 0.0) - wr64) * 32
        if rd + wr < 1e8:            # skip copies and small helpers
            continue
        print(json.dumps({"program": d.split("/")[-2], "kernel": name, "grid": grid,
                          "dispatches": len(next(iter(cs.values()))), "dram_read_GB": round(rd / 1e9, 3),
                          "dram_write_GB": round(wr / 1e9, 3),
                          "rdreq_128B": m.get("TCC_EA0_RDREQ_128B_sum"), "gui_active": m.get("GRBM_GUI_ACTIVE")}))
