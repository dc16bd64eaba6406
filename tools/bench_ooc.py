"""Out-of-core ingest rate: a table whose numeric columns exceed the HBM budget.

Phases (each timed on its own, synchronised):
  ingest   -- ``createDataFrame(pyarrow.Table)`` with ``o3s.storage.hbmBudget`` below the
              table: every numeric column stays on the host, zero copy over the Arrow
              buffers (no device bytes);
  assemble -- ``VectorAssembler`` stages row chunks of the columns through two pinned
              buffer sets (CPU copy of chunk c+1 and its H2D overlap chunk c's kernel),
              assembles them into a SpilledVectorColumn: the resident prefix fills the
              budget, the rest goes back to pinned host rows on a third stream;
  h2d      -- the measured pinned host -> device copy bound on this box (one 4 GiB copy).

The assemble phase moves (n x d x 4) bytes host -> device plus the spilled part of the
bf16 output device -> host; its rate is reported against the H2D bound.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000_000)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--resident-frac", type=float, default=0.25, help="budget as a fraction of the bf16 matrix")
    ap.add_argument("--repeat", type=int, default=1,
                    help="assemble this many times (the previous output dropped first, as when a widget re-runs)")
    a = ap.parse_args()
    import pyarrow as pa
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.frame.spill import SpilledVectorColumn
    from orange3_spark_amd.ml.feature import VectorAssembler
    cuda = torch.cuda.is_available()
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    rng = np.random.default_rng(0)
    names = [f"f{i}" for i in range(a.d)]
    cols = [pa.array(rng.random(a.rows, dtype=np.float32)) for _ in names]
    table = pa.Table.from_arrays(cols, names=names)
    del cols
    in_bytes = a.rows * a.d * 4
    from orange3_spark_amd.ops.glm import padded_width
    out_row = padded_width(a.d) * 2
    budget = int(a.rows * out_row * a.resident_frac)
    s = Session(SessionConf().set("o3s.storage.hbmBudget", str(budget)))
    sync()
    t0 = time.perf_counter()
    df = s.createDataFrame(table)
    sync()
    t_pin = time.perf_counter() - t0
    on_host = df.column_data("f0").data.device.type == "cpu"
    if cuda:
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
    from orange3_spark_amd.frame import spill as SP
    calls = []
    out = col = None
    for _ in range(a.repeat):
        out = col = None                                  # the previous output is dropped
        t0 = time.perf_counter()
        out = VectorAssembler(inputCols=names, outputCol="features").transform(df)
        col = out.column_data("features")
        sync()
        calls.append({"assemble_s": round(time.perf_counter() - t0, 4),
                      "split_s": {k: round(v, 4) if isinstance(v, float) else v
                                  for k, v in SP.LAST_ASSEMBLE_STATS.items()}})
    t_asm = calls[-1]["assemble_s"]
    peak = (torch.cuda.max_memory_allocated() - base) if cuda else 0
    spilled = isinstance(col, SpilledVectorColumn)
    d2h = col.spilled_rows * out_row if spilled else 0
    h2d_gbps = None
    if cuda:
        src = torch.empty(1 << 30, dtype=torch.float32, pin_memory=True)
        dst = torch.empty_like(src, device="cuda")
        dst.copy_(src, non_blocking=True)
        sync()
        t0 = time.perf_counter()
        for _ in range(3):
            dst.copy_(src, non_blocking=True)
        sync()
        h2d_gbps = 3 * src.numel() * 4 / (time.perf_counter() - t0) / 1e9
    asm_gbps = in_bytes / t_asm / 1e9
    print(json.dumps({
        "metric": "out-of-core ingest (host columns -> pinned staging -> streamed VectorAssembler)", "rows": a.rows, "d": a.d,
        "input_GB": round(in_bytes / 1e9, 2), "budget_GB": round(budget / 1e9, 2), "columns_on_host": on_host,
        "spilled": spilled, "resident_rows": col.resident_rows if spilled else len(col),
        "spilled_rows": col.spilled_rows if spilled else 0, "ingest_s": round(t_pin, 3), "assemble_s": round(t_asm, 3),
        "assemble_rows_per_s": a.rows / t_asm, "assemble_input_GBps": round(asm_gbps, 2),
        "d2h_GB": round(d2h / 1e9, 2), "h2d_bound_GBps": None if h2d_gbps is None else round(h2d_gbps, 2),
        "fraction_of_h2d_bound": None if not h2d_gbps else round(asm_gbps / h2d_gbps, 3),
        "device_peak_GB": round(peak / 1e9, 2),
        "calls": calls}), flush=True)


if __name__ == "__main__":
    main()
