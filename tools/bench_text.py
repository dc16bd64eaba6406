"""Tokenizer + HashingTF throughput on synthetic ASCII documents: the device path
(Arrow buffers -> tokenize kernels -> murmur3 over token spans -> CSR) vs the host path
(native C++ tokenizer + python token lists + device murmur3)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd import Session  # noqa: E402
from orange3_spark_amd.ml import feature as F  # noqa: E402
from orange3_spark_amd.ops import text as TX  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--words", type=int, default=50)
    ap.add_argument("--host", action="store_true", help="also time the host tokenizer path")
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    vocab = np.array([f"w{i}" for i in range(50_000)], dtype=object)
    ids = rng.integers(0, len(vocab), (a.docs, a.words))
    docs = [" ".join(vocab[r]) for r in ids]
    s = Session.getOrCreate()
    df = s.createDataFrame(pd.DataFrame({"text": docs}))
    tok, tf = F.Tokenizer(inputCol="text", outputCol="w"), F.HashingTF(inputCol="w", outputCol="tf")
    tf.transform(tok.transform(df.limit(1000))).column_data("tf")
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = tf.transform(tok.transform(df)).column_data("tf")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    res = {"metric": "Tokenizer+HashingTF docs/s (device tokens)", "docs": a.docs, "words_per_doc": a.words,
           "seconds": dt, "docs_per_s": a.docs / dt, "tokens_per_s": a.docs * a.words / dt,
           "nnz": int(out.indptr[-1])}
    # HashingTF alone on the device token column (per-document CSR kernels), best of 5
    words = tok.transform(df)
    col = words.column_data("w")
    best = float("inf")
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        got = tf.transform(words).column_data("tf")
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    ntok = int(col.tok_start.numel())
    res["hashingtf_seconds"] = best
    res["hashingtf_tokens_per_s"] = ntok / best
    # the previous formulation (span buckets + one global sort of (row, bucket) keys)
    torch.cuda.synchronize()
    t = time.perf_counter()
    bucket = TX.murmur3_span_buckets(col, 1 << 18)
    ref = F._buckets_to_csr(bucket, col.doc_offs[1:] - col.doc_offs[:-1], len(col), 1 << 18, False)
    torch.cuda.synchronize()
    res["global_sort_seconds"] = time.perf_counter() - t
    res["same_csr_as_global_sort"] = bool(torch.equal(ref.indptr, got.indptr) and torch.equal(ref.indices, got.indices)
                                          and torch.equal(ref.values, got.values))
    if a.host:
        vals = np.asarray(docs, dtype=object)
        t = time.perf_counter()
        toks = TX.tokenize_lower_ws(vals)
        host = F._terms_to_csr(toks, 1 << 18, s.device, False)
        torch.cuda.synchronize()
        res["host_path_seconds"] = time.perf_counter() - t
        res["same_csr"] = bool(torch.equal(host.indices.cpu(), out.indices.cpu()))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
