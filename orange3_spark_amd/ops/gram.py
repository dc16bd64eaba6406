"""Reductions over the rows as block-batched GEMMs: ``rows_t_matmul(A, B) = A^T B``.

A plain ``A.T @ B`` with A, B of millions of rows and a small output (Gram matrices,
X^T r gradients, per-cluster sums) maps to a GEMM whose output is one or two tiles and
whose K is the row count: hipBLASLt/rocBLAS then run it on one or two workgroups.  fp64 on
one MI355X (tools/bench_gram.py): 4M x 64 X^T X 426 ms -> 0.69 ms as 1024-row batched
GEMMs summed over the batch; X^T v 92 ms -> 0.4 ms; 20M x 256 X^T X 2.1 s -> 41 ms (the
fp64 matrix peak).  Host tensors take the plain product.
"""
from __future__ import annotations

import torch

_BATCH_BYTES = 256 << 20          # bound on the [batches, p, q] partial products


def rows_t_matmul(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A^T B for A [n, p] and B [n, q] (or [n]: returns [p]) of one dtype."""
    vec = B.dim() == 1
    if vec:
        B = B[:, None]
    if not A.is_cuda or A.shape[0] < 8192:
        out = A.T @ B
        return out[:, 0] if vec else out
    n, p = A.shape
    q = B.shape[1]
    bs = 1024 if max(p, q) <= 64 else 4096
    while (n // bs) * p * q * A.element_size() > _BATCH_BYTES:
        bs *= 2
    nb = n // bs
    head = nb * bs
    out = torch.bmm(A[:head].reshape(nb, bs, p).transpose(1, 2), B[:head].reshape(nb, bs, q)).sum(0)
    if head < n:
        out = out + A[head:].T @ B[head:]
    return out[:, 0] if vec else out
