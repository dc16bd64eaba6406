#!/usr/bin/env python
"""Derived (NOT measured) comm budget of exact ALS at N = 2 / 4 / 8 ranks of one node.

Model (models/als.py ``fit_als`` chunked path): each half-iteration solves this rank's
rows of one side in C chunks (``gather_chunks``) and all-gathers each solved chunk into
every rank's slot-layout table while the next chunk solves.  Per half-iteration:

  T_g = table bytes * (N - 1) / N / B        (what every rank receives)
  T_s = the side's solve time at N = 1, / N   (rows split evenly)
  exposed = T_g / C                 if T_g <= T_s   (only the last chunk's transfer)
          = T_g - T_s (1 - 1/C)     otherwise        (transfer-bound: the solve hides part)

B (bytes/s each rank receives in an RCCL all-gather over the 7 xGMI links) is an
assumption until a multi-GPU run measures it: --gbps (default 300, ``O3S_ALS_GATHER_GBPS``).
The per-side solve times come from the N = 1 kernel traces (--user-s / --item-s: seconds
per half-iteration of the full 50M x 5M x 1B config).  Prints a JSON table.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=50_000_000)
    ap.add_argument("--items", type=int, default=5_000_000)
    ap.add_argument("--rank", type=int, default=128)
    ap.add_argument("--user-s", type=float, required=True, help="user-side solve s/half-iteration at N=1")
    ap.add_argument("--item-s", type=float, required=True, help="item-side solve s/half-iteration at N=1")
    ap.add_argument("--other-s", type=float, default=0.0, help="per-iteration non-solve work at N=1 (Gram, eig)")
    ap.add_argument("--gbps", type=float, default=float(os.environ.get("O3S_ALS_GATHER_GBPS", "300")))
    a = ap.parse_args()
    from orange3_spark_amd.models import als as AE
    AE.GATHER_BPS = a.gbps * 1e9
    out = {"assumption": f"all-gather receive rate {a.gbps:.0f} GB/s per rank (not measured)",
           "inputs": {"user_solve_s_n1": a.user_s, "item_solve_s_n1": a.item_s, "other_s_n1": a.other_s}, "rows": []}
    for n in (1, 2, 4, 8):
        row = {"n": n}
        total_exposed = 0.0
        for side, nrows, ts1 in (("user", a.users, a.user_s), ("item", a.items, a.item_s)):
            tbytes = nrows * a.rank * 4
            recv = tbytes * (n - 1) / n
            tg = recv / (a.gbps * 1e9)
            ts = ts1 / n
            c = AE.gather_chunks(nrows, a.rank, n) if n > 1 else 1
            exposed = 0.0 if n == 1 else (tg / c if tg <= ts else tg - ts * (1 - 1 / c))
            total_exposed += exposed
            row[side] = {"recv_GB": round(recv / 1e9, 2), "gather_ms": round(tg * 1e3, 1), "solve_ms": round(ts * 1e3, 1),
                         "chunks": c, "chunk_solve_ms": round(ts / c * 1e3, 2), "exposed_ms": round(exposed * 1e3, 1),
                         "bound": "comm" if tg > ts and n > 1 else "compute"}
        row["iteration_ms"] = round((a.user_s / n + a.item_s / n + a.other_s / n + total_exposed) * 1e3, 1)
        row["exposed_comm_ms"] = round(total_exposed * 1e3, 1)
        out["rows"].append(row)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
