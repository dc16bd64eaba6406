"""String/term ops for HashingTF, FeatureHasher, CountVectorizer, Tokenizer.

Strings live on the host (object arrays); hashing packs them into (offsets, UTF-8 bytes)
and runs MurmurHash3_x86_32 either on the GPU (csrc/text.hip) or in the host C++ library
(csrc/host_text.cpp) -- bit-identical implementations of Spark's term hash (seed 42).
"""
from __future__ import annotations

import ctypes as Ct

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


def tokenize_lower_ws(strings) -> list:
    """Spark Tokenizer semantics: lower-case then split on whitespace (native fast path)."""
    vals = ["" if s is None else s for s in strings]
    offs, data = pack(vals)
    n = len(vals)
    if n == 0:
        return []
    if data.size and int(data.max()) >= 128:        # non-ASCII: Java/Python Unicode lower()
        return [None if s is None else s.lower().split() for s in strings]
    buf = data if data.size else np.zeros(1, np.uint8)
    out = np.empty_like(buf)
    cap = int(data.size // 2 + n + 1)
    ts = np.empty(cap, dtype=np.int64)
    te = np.empty(cap, dtype=np.int64)
    counts = np.empty(n, dtype=np.int64)
    k = N.host().o3s_host_tokenize(offs.ctypes.data, buf.ctypes.data, n, out.ctypes.data, ts.ctypes.data,
                                   te.ctypes.data, cap, counts.ctypes.data)
    if k < 0:
        return [s.lower().split() for s in vals]
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


_ = Ct
