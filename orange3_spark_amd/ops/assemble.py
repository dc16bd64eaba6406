"""VectorAssembler gather kernel (csrc/assemble.hip): numeric / vector columns of any
dtype, with null masks, -> one padded bf16 feature matrix in a single pass, plus per-row
invalid flags and their count (handleInvalid).  CPU tensors are handled by the caller's
torch path (ml/feature.py)."""
from __future__ import annotations


import numpy as np
import torch

from . import _native as N
from .glm import padded_width

_DT = {torch.float64: 0, torch.float32: 1, torch.bfloat16: 2, torch.float16: 3, torch.int64: 4, torch.int32: 5,
       torch.int16: 6, torch.int8: 7, torch.uint8: 8, torch.bool: 9}
_SRC = np.dtype([("ptr", "<u8"), ("valid", "<u8"), ("stride", "<i8"), ("width", "<i4"), ("dtype", "<i4")])
MAX_SOURCES = 512


def supported(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype in _DT and (t.dim() == 1 or (t.dim() == 2 and t.stride(1) == 1))




def _cols_ok(sources) -> bool:
    """Fast-path eligibility (assemble_cols_kernel): plain contiguous [n] float / double
    columns, all of one dtype."""
    dt = sources[0][0].dtype
    return dt in (torch.float32, torch.float64) and all(
        t.dtype == dt and t.dim() == 1 and t.stride(0) == 1 and int(w) == 1 for t, _, w in sources)


def assemble_bf16(sources, n: int, device, path: str = "auto"):
    """``sources``: list of (tensor [n] or [n, >= width] row-major, valid bool [n] or None,
    width).  Returns (bf16 [n, ld] zero padded, uint8 invalid flags [n], invalid count).
    ``path``: "auto" (column-window kernel when every source is a plain float / double
    column, else the generic gather), "cols" or "generic"."""
    if not sources or len(sources) > MAX_SOURCES:
        raise ValueError(f"assemble needs 1..{MAX_SOURCES} source columns")
    recs = np.zeros(len(sources), dtype=_SRC)
    colmap = []
    keep = []
    for i, (t, valid, width) in enumerate(sources):
        if not supported(t) or t.shape[0] != n:
            raise TypeError("assemble sources must be cuda tensors with one row per frame row")
        if valid is not None:
            valid = valid.to(device=t.device).contiguous()
            valid = valid.view(torch.uint8) if valid.dtype == torch.bool else valid.to(torch.uint8)
            keep.append(valid)
        keep.append(t)
        recs[i] = (t.data_ptr(), 0 if valid is None else valid.data_ptr(),
                   1 if t.dim() == 1 else t.stride(0), int(width), _DT[t.dtype])
        colmap += [(i, e) for e in range(int(width))]
    D = len(colmap)
    ld = padded_width(D)
    lib = N.kernels()
    assert lib.o3s_assemble_src_size() == _SRC.itemsize
    src_d, map_d = N.upload_many(device, recs.view(np.uint8), np.asarray(colmap, dtype=np.int32).reshape(-1))
    out = torch.empty((n, ld), dtype=torch.bfloat16, device=device)
    bad = torch.empty(n, dtype=torch.uint8, device=device)
    nbad = torch.zeros(1, dtype=torch.int32, device=device)
    cols = path == "cols" or (path == "auto" and _cols_ok(sources))
    if cols:
        if not _cols_ok(sources):
            raise ValueError("the column-window assembler needs plain float / double columns of one dtype")
        rows, per_cu = 256, 4                # 256-row blocks (assemble_cols_kernel)
        grid = max(1, min(N.num_cus(torch.device(device)) * per_cu * 2, -(-n // rows)))
        if grid >= 8:
            grid -= grid % 8          # the kernel's XCD-aware block walk wants G % 8 == 0
        N.check(lib.o3s_assemble_cols(src_d.data_ptr(), _DT[sources[0][0].dtype], D, ld, n, out.data_ptr(), 0,
                                      bad.data_ptr(), nbad.data_ptr(), grid, N.stream_of(out)), "assemble_cols")
        del keep
        return out, bad, nbad, D
    grid = max(1, min(N.num_cus(torch.device(device)) * 8, -(-n // 64)))
    N.check(lib.o3s_assemble(src_d.data_ptr(), len(sources), map_d.data_ptr(), D, ld, n, out.data_ptr(), 0,
                             bad.data_ptr(), nbad.data_ptr(), grid, N.stream_of(out)), "assemble")
    del keep
    return out, bad, nbad, D
