"""ctypes binding of the in-tree gfx950 kernel library (``_lib/libo3s_kernels.so``).

Policy ("fail loudly"): on a machine with a visible GPU every op dispatches to the HIP
kernels; if the library is missing or does not load there, :func:`kernels` raises
instead of silently using a PyTorch fallback.  The PyTorch reference implementations
are only used for CPU tensors (tests, the CPU plumbing config) -- see
``ops/__init__.py``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import torch

from ..runtime.faults import O3SError
from . import build as _build

_LOCK = threading.Lock()
_LIB = None
_HOST = None

c_i64, c_i32, c_u32, c_f32, c_f64 = C.c_int64, C.c_int, C.c_uint32, C.c_float, C.c_double
c_vp = C.c_void_p

# name -> argtypes (every kernel entry point returns int: 0 = ok, <0 arg error, >0 hipError)
_SIGS: dict[str, list] = {
    "o3s_glm_layout": [c_i64, C.POINTER(c_i32), C.POINTER(c_i32)],
    "o3s_glm_grad": [c_i32, c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_u32, c_i64,
                     c_vp, c_f32, c_vp, c_i32, c_vp, c_i32, c_vp],
    "o3s_glm_grad_mixed": [c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_u32, c_i64, c_i64,
                           c_vp, c_i32, c_vp, c_i32, c_i64, c_vp, c_u32, c_u32, c_i32, c_vp],
    "o3s_glm_stats_mixed": [c_vp, c_i64, c_i64, c_vp, c_vp, c_u32, c_i64, c_i64, c_vp, c_i32, c_vp, c_i32, c_vp],
    "o3s_bin_features": [c_vp, c_i64, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp],
    "o3s_u8_transpose": [c_vp, c_i64, c_i32, c_vp, c_vp],
    "o3s_slab_range_sum": [c_vp, c_i32, c_i64, c_vp, c_vp, c_i32, c_vp, c_vp],
    "o3s_tree_leaf_apply": [c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp],
    "o3s_ftf": [c_vp, c_i64, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp],
    "o3s_als_gram": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp],
    "o3s_csr_glm": [c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp],
    "o3s_csc_colsum": [c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp],
    "o3s_csc_piece": [],
    "o3s_tokenize": [c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "o3s_murmur3_spans": [c_vp, c_vp, c_vp, c_i64, c_u32, c_i64, c_vp, c_vp],
    "o3s_tree_partition": [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32,
                           c_vp, c_vp, c_vp, c_vp, c_vp],
    "o3s_glm_sgd_update": [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_f64, c_f64, c_i32, c_vp, c_vp, c_vp],
    "o3s_glm_sgd_update_dev": [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_f64, c_vp, c_f64, c_f64, c_i32, c_vp, c_vp,
                               c_i64, c_vp, c_vp],
    "o3s_synth_glm": [c_vp, c_i64, c_i64, c_vp, c_u32, c_i64, c_vp, c_f32, c_i32, c_vp],
    "o3s_glm_margin": [c_vp, c_i64, c_i64, c_vp, c_f32, c_vp, c_i32, c_vp],
    "o3s_glm_colstats": [c_i32, c_vp, c_i64, c_i64, c_vp, c_u32, c_i64, c_vp, c_i32, c_vp, c_vp],
    "o3s_bin_sums": [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp],
    "o3s_glm_softmax": [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp],
    "o3s_kmeans_assign": [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp],
    "o3s_kmeans_screen2": [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32, C.c_float, C.c_float,
                           C.c_float, C.c_float, C.c_float, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp,
                           c_vp, c_vp],
    "o3s_kmeans_presplit": [c_vp, c_i64, c_i64, c_i32, C.c_float, c_vp, c_vp, c_vp],
    "o3s_kmeans_moments": [c_vp, c_i64, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp],
    "o3s_kmeans_cost": [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp],
    "o3s_kmeans_bounds": [c_vp, c_vp, c_i64, c_vp, C.c_float, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp],
    "o3s_kmeans_update_ws": [c_i32, c_i32, c_i32, C.POINTER(c_i64), C.POINTER(c_i64), C.POINTER(c_i32)],
    "o3s_murmur3_terms": [c_vp, c_vp, c_i64, c_u32, c_i64, c_vp, c_vp, c_vp],
    "o3s_als_init": [c_i64, c_i64, c_i32, c_u32, c_i32, c_vp, c_vp],
    "o3s_als_cg": [c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "o3s_als_pass": [c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp],
    "o3s_tree_hist_lds": [c_i32, c_i32, c_i32, c_i32],
    "o3s_hash_uniform": [c_vp, c_i64, c_i64, c_u32, c_u32, c_i32, c_f64, c_vp, c_vp, c_vp],
    "o3s_tree_final_level": [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_i32, c_vp],
    "o3s_forest_weights": [c_vp, c_i64, c_vp, c_i32, c_vp, c_i32, c_f32, c_vp, c_vp, c_vp],
    "o3s_tree_sibling": [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp],
    "o3s_tree_part_dest": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp],
    "o3s_gbt_grad_loss": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i32, c_vp],
    "o3s_gbt_leaf_pass": [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32,
                          c_vp, c_vp, c_vp, c_i32, c_vp],
    "o3s_tree_split": [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_f64, c_f64, c_f64, c_vp, c_vp, c_vp],
    "o3s_tree_hist": [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32,
                      c_vp],
    "o3s_eval_grid": [c_i64],
    "o3s_regression_stats": [c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_i64, c_vp, c_vp, c_vp],
    "o3s_confusion": [c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp],
    "o3s_score_hist": [c_vp, c_i32, c_i64, c_vp, c_i32, c_vp, c_i32, c_i64, c_f64, c_f64, c_i32, c_vp, c_vp],
    "o3s_als_wood_kn": [c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp],
    "o3s_als_wood_timed": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp],
    "o3s_hashing_tf": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_u32, c_i64, c_vp, c_vp, c_vp, c_vp, c_i32,
                       c_vp, c_vp, c_vp],
    "o3s_als_dense_wave_dbg": [c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp],
    "o3s_bin_features2": [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp, c_i64, c_vp],
    "o3s_kmeanspp": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "o3s_als_dense_wave_timed": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp],
    "o3s_als_dense_wave": [c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp],
    "o3s_als_dense_wave_gd": [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp],
    "o3s_als_exact_max_small": [],
    "o3s_als_rotate": [c_i32, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp],
    "o3s_als_rotate_to": [c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_i32, c_vp],
    "o3s_assemble": [c_vp, c_i32, c_vp, c_i32, c_i32, c_i64, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp],
    "o3s_assemble_src_size": [],
    "o3s_assemble_cols": [c_vp, c_i32, c_i32, c_i32, c_i64, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp],
    "o3s_kmeans_update": [c_vp, c_i64, c_i64, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp],
    "o3s_gather_probe": [c_vp, c_i32, c_vp, c_i64, c_i32, c_vp, c_vp],
}


class NativeError(O3SError):
    """A native kernel launch was rejected (bad shape/arguments) or failed."""


def lib_path() -> Path:
    # O3S_KERNEL_LIB: an alternative build of the library (A/B timing tools only)
    alt = os.environ.get("O3S_KERNEL_LIB")
    return Path(alt) if alt else _build.KERNEL_LIB


def _load():
    global _LIB
    path = lib_path()
    if not path.exists() and os.environ.get("O3S_AUTOBUILD", "1") == "1":
        _build.build()
    if not path.exists():
        raise NativeError(f"kernel library missing: {path} (run python -m orange3_spark_amd.ops.build)")
    lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
    for name, argt in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = argt
        fn.restype = C.c_int
    _LIB = lib
    return lib


def kernels():
    """Return the loaded kernel library (raises NativeError if it cannot be loaded)."""
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        return _load()


_HOST_SIGS: dict[str, list] = {
    "o3s_host_murmur3": [c_vp, c_vp, c_i64, c_u32, c_i64, c_vp, c_vp],
    "o3s_host_tokenize": [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp],
    "o3s_host_pav": [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp],
    "o3s_host_ascii_lengths": [c_vp, c_i64, c_vp, c_vp],
    "o3s_host_ascii_pack": [c_vp, c_i64, c_vp, c_vp, c_i32],
}
_HOST_RET = {"o3s_host_tokenize": C.c_int64, "o3s_host_pav": C.c_int64, "o3s_host_ascii_lengths": C.c_int64}


def host():
    """Host C++ runtime library (text hashing/tokenizing, PAV); built with the kernels."""
    global _HOST
    if _HOST is not None:
        return _HOST
    with _LOCK:
        if _HOST is None:
            path = _build.HOST_LIB
            if not path.exists():
                _build.build()
            lib = C.CDLL(str(path))
            for name, argt in _HOST_SIGS.items():
                fn = getattr(lib, name)
                fn.argtypes = argt
                fn.restype = _HOST_RET.get(name)
            _HOST = lib
    return _HOST


PRELOAD_TAGS = ("glm", "trees", "kmeans", "als", "als_dense", "als_exact", "assemble", "binsum", "eval",
                "sampling", "sparse", "text", "probe")


def preload(tags=PRELOAD_TAGS) -> dict:
    """Load the gfx950 code objects of the given kernel files on the current device without
    launching anything (``O3S_PRELOAD`` in ``csrc/common.h``); seconds per file."""
    import time
    lib = kernels()
    out = {}
    for tag in tags:
        fn = getattr(lib, f"o3s_preload_{tag}", None)
        if fn is None:
            continue
        fn.restype = C.c_int
        t = time.perf_counter()
        rc = fn()
        if rc != 0:
            raise NativeError(f"o3s_preload_{tag}: hipError {rc}")
        out[tag] = round(time.perf_counter() - t, 5)
    return out


def available() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def upload(arr, dev) -> torch.Tensor:
    """Host array -> device tensor WITHOUT stalling the host: staged through (cached)
    pinned memory and copied non_blocking on the current stream.  A pageable copy
    blocks the host until the stream has drained, so every small plan upload of a
    launch-bound loop (tree levels) would leave the GPU idle while Python catches up;
    PyTorch's caching host allocator keeps the pinned block alive until the copy ran."""
    import numpy as np
    t = torch.from_numpy(np.ascontiguousarray(arr))
    dev = torch.device(dev)
    if dev.type != "cuda":
        return t.to(dev)
    p = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    p.copy_(t)
    return p.to(dev, non_blocking=True)


def upload_many(dev, *arrays) -> list:
    """Several small host arrays -> device tensors through ONE staged copy: the arrays
    are packed (8-byte aligned) into one pinned buffer and the device tensors are typed
    views into its device copy."""
    import numpy as np
    arrs = [np.ascontiguousarray(a) for a in arrays]
    offs, total = [], 0
    for a in arrs:
        offs.append(total)
        total += (a.nbytes + 7) // 8 * 8
    buf = np.zeros(max(total, 8), dtype=np.uint8)
    for a, o in zip(arrs, offs):
        buf[o:o + a.nbytes] = a.view(np.uint8).reshape(-1)
    d = upload(buf, dev)
    out = []
    for a, o in zip(arrs, offs):
        dt = torch.from_numpy(np.zeros(0, dtype=a.dtype)).dtype
        out.append(d[o:o + a.nbytes].view(dt).view(a.shape))
    return out


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def check(rc: int, what: str) -> None:
    """Validate a native launch's return code (+ fault injection / launch-blocking mode)."""
    from ..runtime import faults
    faults.INJECTOR.hit("kernel")
    if rc != 0:
        raise NativeError(f"{what} failed with code {rc}")
    if faults.launch_blocking() and torch.cuda.is_available():
        try:
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 - surfaces async HIP faults at the launching call
            raise faults.DeviceError(what, e) from e


def num_cus(device: torch.device) -> int:
    try:
        return torch.cuda.get_device_properties(device).multi_processor_count
    except Exception:
        return 256


def grid_for(device: torch.device, work_items: int, per_block: int, blocks_per_cu: int = 8) -> int:
    """Grid for a streaming kernel: enough blocks to fill every CU, capped (Guideline 11)."""
    need = max(1, (work_items + per_block - 1) // per_block)
    return int(max(1, min(need, num_cus(device) * blocks_per_cu)))
