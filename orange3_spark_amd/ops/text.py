"""String/term ops for HashingTF, FeatureHasher, CountVectorizer, Tokenizer.

Strings live on the host (object arrays); hashing packs them into (offsets, UTF-8 bytes)
and runs MurmurHash3_x86_32 either on the GPU (csrc/text.hip) or in the host C++ library
(csrc/host_text.cpp) -- bit-identical implementations of Spark's term hash (seed 42).
"""
from __future__ import annotations

import ctypes as Ct
import os
import re

import numpy as np
import torch

from . import _native as N

SPARK_SEED = 42


def pack(strings) -> tuple[np.ndarray, np.ndarray]:
    enc = [s.encode("utf-8") for s in strings]
    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    data = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, dtype=np.uint8)
    return offs, data


def murmur3_buckets(strings, num_buckets: int, device=None, seed: int = SPARK_SEED):
    """(hash int32 [n], bucket int64 [n]) for each string."""
    offs, data = pack(strings)
    n = len(offs) - 1
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda" and n:
        o = torch.from_numpy(offs).to(dev)
        b = torch.from_numpy(data.copy() if data.size else np.zeros(1, np.uint8)).to(dev)
        h = torch.empty(n, dtype=torch.int32, device=dev)
        k = torch.empty(n, dtype=torch.int64, device=dev)
        N.check(N.kernels().o3s_murmur3_terms(o.data_ptr(), b.data_ptr(), n, seed, num_buckets, h.data_ptr(),
                                              k.data_ptr(), N.stream_of(o)), "murmur3")
        return h, k
    h = np.empty(n, dtype=np.int32)
    k = np.empty(n, dtype=np.int64)
    if n:
        buf = data if data.size else np.zeros(1, np.uint8)
        N.host().o3s_host_murmur3(offs.ctypes.data, buf.ctypes.data, n, seed, num_buckets, h.ctypes.data,
                                  k.ctypes.data)
    return torch.from_numpy(h), torch.from_numpy(k)


_WS = re.compile(r"[ \t\n\x0b\f\r]")


def spark_split(s: str) -> list:
    """Java ``s.split("\\s")``: every single whitespace char separates (runs give empty
    tokens), trailing empty tokens dropped, "" -> [""] (Spark Tokenizer after lower-case)."""
    if s == "":
        return [""]
    parts = _WS.split(s)
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def tokenize_lower_ws(strings) -> list:
    """Spark Tokenizer semantics (lower-case, then ``split("\\s")``; native fast path for
    ASCII columns, Python for non-ASCII text where Unicode lower-casing is needed)."""
    vals = ["" if s is None else s for s in strings]
    offs, data = pack(vals)
    n = len(vals)
    if n == 0:
        return []
    if data.size and int(data.max()) >= 128:        # non-ASCII: Java/Python Unicode lower()
        return [None if s is None else spark_split(s.lower()) for s in strings]
    buf = data if data.size else np.zeros(1, np.uint8)
    out = np.empty_like(buf)
    cap = int(data.size + n + 1)                     # <= one token per byte + one per string
    ts = np.empty(cap, dtype=np.int64)
    te = np.empty(cap, dtype=np.int64)
    counts = np.empty(n, dtype=np.int64)
    k = N.host().o3s_host_tokenize(offs.ctypes.data, buf.ctypes.data, n, out.ctypes.data, ts.ctypes.data,
                                   te.ctypes.data, cap, counts.ctypes.data)
    if k < 0:
        return [None if s is None else spark_split(s.lower()) for s in strings]
    raw = out.tobytes()
    res, j = [], 0
    for i in range(n):
        c = int(counts[i])
        res.append([raw[ts[j + q]:te[j + q]].decode("utf-8", "replace") for q in range(c)])
        j += c
    for i, s in enumerate(strings):
        if s is None:
            res[i] = None
    return res


def arrow_strings(values):
    """(offsets int64 [n+1], UTF-8 bytes uint8, valid bool [n] | None) of an object array of
    str/None, converted in C by pyarrow (no per-string Python work)."""
    import pyarrow as pa
    arr = pa.array(values, type=pa.large_string(), from_pandas=True)
    validity, obuf, dbuf = arr.buffers()
    n = len(arr)
    offs = np.frombuffer(obuf, dtype=np.int64, count=n + 1, offset=8 * arr.offset)
    base = int(offs[0])
    data = np.frombuffer(dbuf, dtype=np.uint8) if dbuf is not None else np.zeros(0, np.uint8)
    data = data[base: int(offs[-1])]
    valid = None
    if arr.null_count:
        valid = ~np.asarray(arr.is_null().to_numpy(zero_copy_only=False), dtype=bool)
    return offs - base, data, valid


def pack_strings(values):
    """(offsets int64 [n+1], bytes uint8, valid bool [n] | None, ascii) of an object array of
    str / None.  Compact ASCII columns (the common case) are packed by the host runtime
    (csrc/host_strings.cpp: a length pass, then a threaded copy of each string's bytes,
    GIL released) -- ascii=True; anything else goes through pyarrow -- ascii=None (unknown:
    the caller checks the bytes).

    The native passes read the str objects with the GIL released, so they run over a
    private snapshot of the column (``np.array(..., copy=True)``: a new array holding its
    own reference to every object, taken under the GIL).  Another thread that replaces an
    element of the caller's array meanwhile can then neither free an object the passes
    read nor make the length pass and the copy pass see different strings."""
    vals = np.array(values, dtype=object, copy=True)
    n = vals.shape[0]
    if vals.ndim == 1 and vals.flags.c_contiguous and n:
        lib = N.host()
        offs = np.empty(n + 1, dtype=np.int64)
        valid = np.empty(n, dtype=np.uint8)
        tot = lib.o3s_host_ascii_lengths(vals.ctypes.data, n, offs.ctypes.data, valid.ctypes.data)
        if tot >= 0:
            data = np.empty(max(tot, 1), dtype=np.uint8)
            lib.o3s_host_ascii_pack(vals.ctypes.data, n, offs.ctypes.data, data.ctypes.data,
                                    min(16, os.cpu_count() or 1))
            v = valid.view(bool)
            return offs, data[:tot], (None if v.all() else v.copy()), True
    offs, data, valid = arrow_strings(vals)
    return offs, data, valid, None


def device_tokenize(values, device, min_rows: int = 1):
    """Spark Tokenizer on the GPU for an ASCII string column: returns a
    :class:`~orange3_spark_amd.frame.column.DeviceTokensColumn` (tokens stay on the device
    as spans of the lower-cased byte buffer), or None when the column needs the host path
    (non-ASCII text, CPU device, or fewer than ``min_rows`` rows)."""
    from ..frame.column import DeviceTokensColumn
    dev = torch.device(device)
    if dev.type != "cuda" or len(values) < min_rows:
        return None
    offs, data, valid, ascii_ = pack_strings(values)
    if not ascii_ and data.size and int(data.max()) >= 128:
        return None
    n = len(offs) - 1
    o = torch.from_numpy(np.ascontiguousarray(offs)).to(dev)
    b = torch.from_numpy(data if data.size and data.flags.writeable else
                         (data.copy() if data.size else np.zeros(1, np.uint8))).to(dev)
    lib = N.kernels()
    st = N.stream_of(o)
    counts = torch.empty(n, dtype=torch.int64, device=dev)
    N.check(lib.o3s_tokenize(0, o.data_ptr(), b.data_ptr(), n, counts.data_ptr(), None, None, None, None, st),
            "tokenize_count")
    if valid is not None:
        counts.masked_fill_(torch.from_numpy(~valid).to(dev), 0)
    doc_offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=doc_offs[1:])
    ntok = int(doc_offs[-1])
    low = torch.empty_like(b)
    ts = torch.empty(max(ntok, 1), dtype=torch.int64, device=dev)
    te = torch.empty(max(ntok, 1), dtype=torch.int64, device=dev)
    # null rows hold "" in the Arrow buffers; their masked count of 0 makes emit skip them
    N.check(lib.o3s_tokenize(1, o.data_ptr(), b.data_ptr(), n, None, doc_offs.data_ptr(), low.data_ptr(),
                             ts.data_ptr(), te.data_ptr(), st), "tokenize_emit")
    vt = None if valid is None else torch.from_numpy(valid).to(dev)
    return DeviceTokensColumn(doc_offs, ts[:ntok], te[:ntok], low, vt)


def murmur3_span_buckets(tok, num_buckets: int, seed: int = SPARK_SEED) -> torch.Tensor:
    """Bucket (int64) of every token of a DeviceTokensColumn (Spark HashingTF hash)."""
    ntok = int(tok.tok_start.numel())
    out = torch.empty(ntok, dtype=torch.int64, device=tok.data.device)
    N.check(N.kernels().o3s_murmur3_spans(tok.tok_start.data_ptr(), tok.tok_end.data_ptr(), tok.data.data_ptr(),
                                          ntok, seed, num_buckets, out.data_ptr(), N.stream_of(out)),
            "murmur3_spans")
    return out


def hashing_tf_csr(tok, num_buckets: int, binary: bool, seed: int = SPARK_SEED):
    """Spark HashingTF of a DeviceTokensColumn straight to CSR (indptr int64, indices int32,
    values fp64), per document on the GPU (csrc/text.hip ``hashing_tf_*_kernel``: one wave
    per document, bitonic sort + run counting in registers / LDS; no global sort).
    Documents of more than 4096 tokens are counted by a torch sort of their own buckets."""
    dev = tok.data.device
    n = len(tok)
    ntok = int(tok.tok_start.numel())
    lib = N.kernels()
    st = N.stream_of(tok.doc_offs)
    tmp_idx = torch.empty(max(ntok, 1), dtype=torch.int32, device=dev)
    tmp_cnt = torch.empty(max(ntok, 1), dtype=torch.int32, device=dev)
    nnz = torch.zeros(n, dtype=torch.int64, device=dev)
    args = (tok.doc_offs.data_ptr(), tok.tok_start.data_ptr(), tok.tok_end.data_ptr(), tok.data.data_ptr())
    N.check(lib.o3s_hashing_tf(0, *args, None, n, seed, num_buckets, tmp_idx.data_ptr(), tmp_cnt.data_ptr(),
                               nnz.data_ptr(), None, 0, None, None, st), "hashing_tf")
    big = torch.nonzero(nnz < 0).reshape(-1)
    if big.numel():
        huge = big[nnz[big] == -2]
        large = big[nnz[big] == -1].contiguous()
        if large.numel():
            N.check(lib.o3s_hashing_tf(1, *args, large.data_ptr(), large.numel(), seed, num_buckets,
                                       tmp_idx.data_ptr(), tmp_cnt.data_ptr(), nnz.data_ptr(), None, 0, None, None,
                                       st), "hashing_tf_large")
        for d in huge.tolist():                     # > 4096 tokens: rare, one sort each
            a, b = int(tok.doc_offs[d]), int(tok.doc_offs[d + 1])
            sub = type(tok)(torch.tensor([0, b - a], device=dev), tok.tok_start[a:b], tok.tok_end[a:b], tok.data)
            u, c = torch.unique(murmur3_span_buckets(sub, num_buckets, seed), return_counts=True)
            tmp_idx[a:a + u.numel()] = u.to(torch.int32)
            tmp_cnt[a:a + u.numel()] = c.to(torch.int32)
            nnz[d] = u.numel()
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nnz, 0, out=indptr[1:])
    total = int(indptr[-1])
    idx = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(total, 1), dtype=torch.float64, device=dev)
    N.check(lib.o3s_hashing_tf(2, *args, None, n, seed, num_buckets, tmp_idx.data_ptr(), tmp_cnt.data_ptr(),
                               nnz.data_ptr(), indptr.data_ptr(), int(bool(binary)), idx.data_ptr(), val.data_ptr(),
                               st), "hashing_tf_compact")
    return indptr, idx[:total], val[:total]
