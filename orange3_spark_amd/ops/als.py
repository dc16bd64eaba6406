"""ALS ratings passes: gfx950 kernel (csrc/als.hip) with a PyTorch reference.

mode 0 (matvec): out[u] = sum_j coef_j * (F[c_j] . V[u]) * F[c_j]
mode 1 (rhs)   : out[u] = sum_j coef_j * F[c_j]
"""
from __future__ import annotations

import os

import torch

from . import _native as N
from ..runtime.tracing import trace


def pass_torch(mode, indptr, cols, coef, F, V):
    """``indptr`` may be a row-range view of a larger CSR (absolute offsets into cols/coef,
    as the kernel reads them)."""
    n = indptr.numel() - 1
    R = F.shape[1]
    base, end = int(indptr[0]), int(indptr[-1])
    if base or end != cols.numel():
        cols, coef, indptr = cols[base:end], coef[base:end], indptr - base
    rows = torch.repeat_interleave(torch.arange(n, device=F.device), indptr[1:] - indptr[:-1])
    Fg = F[cols.long()].to(torch.float64)
    s = coef.to(torch.float64)
    if mode == 0:
        s = s * (Fg * V.to(torch.float64)[rows]).sum(1)
    out = torch.zeros((n, R), dtype=torch.float64, device=F.device).index_add_(0, rows, Fg * s[:, None])
    return out.to(F.dtype)


def pass_(mode, indptr, cols, coef, F, V=None):
    n = indptr.numel() - 1
    R = F.shape[1]
    if F.is_cuda and F.dtype == torch.float32 and R <= 512:
        out = torch.empty((n, R), dtype=torch.float32, device=F.device)
        Fc = F.contiguous()
        Vc = None if V is None else V.contiguous().float()
        N.check(N.kernels().o3s_als_pass(mode, indptr.data_ptr(), cols.data_ptr(), coef.data_ptr(), n,
                                         Fc.data_ptr(), R, N.ptr(Vc), out.data_ptr(), None, None,
                                         N.stream_of(Fc)), "als_pass")
        return out
    return pass_torch(mode, indptr, cols, coef, F, V)


def pass_both(indptr, cols, coef, F, V, coef2):
    """(matvec with coef at V, rhs with coef2) in ONE gather pass over the ratings."""
    n = indptr.numel() - 1
    R = F.shape[1]
    if F.is_cuda and F.dtype == torch.float32 and R <= 512:
        out = torch.empty((n, R), dtype=torch.float32, device=F.device)
        out2 = torch.empty((n, R), dtype=torch.float32, device=F.device)
        Fc = F.contiguous()
        N.check(N.kernels().o3s_als_pass(2, indptr.data_ptr(), cols.data_ptr(), coef.data_ptr(), n, Fc.data_ptr(),
                                         R, V.contiguous().float().data_ptr(), out.data_ptr(), coef2.data_ptr(),
                                         out2.data_ptr(), N.stream_of(Fc)), "als_pass2")
        return out, out2
    return pass_torch(0, indptr, cols, coef, F, V), pass_torch(1, indptr, cols, coef2, F, None)


def cg_kernel_ok(F: torch.Tensor) -> bool:
    return F.is_cuda and F.dtype == torch.float32 and F.shape[1] <= 512


def cg_init(x, ax, pf, rhs, lam):
    """Fused CG start (als_cg_kernel mode 0): returns (r, p, rs) for
    r = rhs - (ax + pf + lam*x)."""
    n, R = x.shape
    r = torch.empty_like(x)
    p = torch.empty_like(x)
    rs = torch.empty(n, dtype=torch.float32, device=x.device)
    N.check(N.kernels().o3s_als_cg(0, n, R, x.data_ptr(), r.data_ptr(), p.data_ptr(), ax.data_ptr(), N.ptr(pf),
                                   rhs.data_ptr(), lam.data_ptr(), rs.data_ptr(), N.stream_of(x)), "als_cg_init")
    return r, p, rs


def cg_step(x, r, p, ap, pf, lam, rs):
    """Fused CG step (als_cg_kernel mode 1): updates x, r, p, rs in place."""
    n, R = x.shape
    N.check(N.kernels().o3s_als_cg(1, n, R, x.data_ptr(), r.data_ptr(), p.data_ptr(), ap.data_ptr(), N.ptr(pf),
                                   None, lam.data_ptr(), rs.data_ptr(), N.stream_of(x)), "als_cg_step")


def gram_ok(F: torch.Tensor) -> bool:
    R = F.shape[1]
    return F.is_cuda and F.dtype == torch.float32 and R % 32 == 0 and 32 <= R <= 128


def dense_solve(indptr, cols, w, b, F, FtF, lam, batch_bytes: int = 1 << 30) -> torch.Tensor:
    """Exact per-row normal-equation solves: ``als_gram_kernel`` (MFMA) forms
    A_u = FtF + sum w y y^T + lam_u I and b_u for a batch of rows, a batched Cholesky
    (rocSOLVER via torch.linalg.cholesky_ex) solves them; rows whose fp32 factorisation
    fails are re-solved in fp64."""
    n = indptr.numel() - 1
    R = F.shape[1]
    dev = F.device
    x = torch.empty((n, R), dtype=torch.float32, device=dev)
    bs = max(1, min(n, batch_bytes // (R * R * 4)))
    Fc = F.contiguous()
    Gc = None if FtF is None else FtF.contiguous().float()
    lib = N.kernels()
    A = torch.empty((bs, R, R), dtype=torch.float32, device=dev)
    bv = torch.empty((bs, R), dtype=torch.float32, device=dev)
    for r0 in range(0, n, bs):
        m = min(bs, n - r0)
        N.check(lib.o3s_als_gram(indptr.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(), Fc.data_ptr(), R,
                                 N.ptr(Gc), lam.data_ptr(), r0, m, A.data_ptr(), bv.data_ptr(), N.stream_of(Fc)),
                "als_gram")
        L, info = torch.linalg.cholesky_ex(A[:m])
        xs = torch.cholesky_solve(bv[:m, :, None], L)[:, :, 0]
        bad = info != 0
        if bool(bad.any()):
            Ad = A[:m][bad].double()
            Ad = Ad + 1e-12 * torch.eye(R, dtype=torch.float64, device=dev)[None]
            xs[bad] = torch.linalg.solve(Ad, bv[:m][bad].double()[:, :, None])[:, :, 0].float()
        x[r0:r0 + m] = xs
    return x


EXACT_RANKS = (32, 64, 96, 128)
# eigenbasis dense solves with G = diag(eig) passed as a vector (no 40 KB G image in LDS,
# so a 4-step gather ring at rank 128); O3S_ALS_DENSE_GDIAG=0: the full-G build (A/B)
DENSE_GDIAG = os.environ.get("O3S_ALS_DENSE_GDIAG", "1") != "0"

# Long rows (more than 32 ratings, or lam_u = 0) take als_dense_wave_kernel
# (csrc/als_dense.hip): one wave per row, four independent waves per CU, factor rows
# gathered by an LDS-DMA ring that streams across the rows of a wave, rows listed longest
# first.  625K items x 200 ratings at rank 128: 34.0 ms against 45.2 ms for the round-4
# block-per-row kernel (profiles/als_dense_wave_r5.json).  Rows with <= 16 / 17..24 / 25..32
# ratings take Woodbury launches sized to them (16 x 16 S on 16x16x4 MFMAs for the first).


_FTF_WS: dict = {}


def ftf(F: torch.Tensor) -> torch.Tensor:
    """F^T F (fp64 [R, R]) of a device fp32 table with unit column stride and R <= 128
    (``ftf_kernel`` + ``ftf_reduce_kernel``: bitwise reproducible for a given shape)."""
    n, R = F.shape
    nt = (R + 31) // 32
    nl = nt * (nt + 1) // 2
    nwaves = max(4, min(2048, (-(-n // 4096) + 3) // 4 * 4))
    need = nwaves * nl * 1024
    ws = _FTF_WS.get(F.device)
    if ws is None or ws.numel() < need:
        ws = torch.empty(max(need, 2048 * 10 * 1024 if n >= (1 << 22) else need), dtype=torch.float32,
                         device=F.device)
        _FTF_WS[F.device] = ws
    out = torch.empty((R, R), dtype=torch.float64, device=F.device)
    N.check(N.kernels().o3s_ftf(F.data_ptr(), n, F.stride(0), R, nwaves, ws.data_ptr(), out.data_ptr(),
                                N.stream_of(F)), "ftf")
    return out


def exact_kernel_ok(F: torch.Tensor) -> bool:
    """Any rank up to 128 runs on the kernels: ranks between the compiled sizes are padded
    with zero factor columns (see :func:`exact_solve`)."""
    return F.is_cuda and F.dtype == torch.float32 and 0 < F.shape[1] <= EXACT_RANKS[-1] and F.is_contiguous()


def _padded_rank(R: int) -> int:
    return next(r for r in EXACT_RANKS if r >= R)


class _PadCache:
    """Zero-padded copy of a factor table (rank R -> the next compiled size), reused by
    the calls of one half-iteration; keyed like _EigCache on the tensor and its version."""

    def __init__(self):
        self.key = None
        self.val = None

    def get(self, F, Rp):
        import weakref
        key = (F._version, tuple(F.shape), Rp)
        if self.key is not None and self.key[0]() is F and self.key[1] == key:
            return self.val
        Fp = torch.zeros((F.shape[0], Rp), dtype=F.dtype, device=F.device)
        Fp[:, :F.shape[1]] = F
        self.key, self.val = (weakref.ref(F), key), Fp
        return Fp

    def clear(self):
        self.key = self.val = None


PAD_CACHE = _PadCache()


class _EigCache:
    """Eigendecomposition of G and the rotated table F Q for the Woodbury rows, kept for
    the calls of one half-iteration (the chunked path solves its rows in several calls
    against the same F and G).  Keyed on the tensors themselves (weak references plus
    their version counters), so an in-place update or a new table recomputes."""

    def __init__(self):
        self.key = None
        self.val = None
        # set by fit_als for multi-rank eigenbasis fits: (eig, Q) then come from rank 0 --
        # every rank's tables must live in the SAME basis, and LAPACK on different ranks
        # (different CPUs / BLAS dispatch) may pick different signs or degenerate vectors
        self.comm = None

    def get(self, F, G, need_fq: bool, shared: bool = False):
        import weakref
        key = (F._version, G._version, tuple(F.shape))
        if (self.key is not None and self.key[0]() is F and self.key[1]() is G and self.key[2] == key
                and (self.val[2] is not None or not need_fq)):
            return self.val
        # the rank x rank eigendecomposition runs on the host (LAPACK, fp64): 1.4 ms for
        # R = 128 against 2.2 ms for torch.linalg.eigh on the GPU, whose first call in a
        # process also pays ~125 ms of solver start-up (tools/probe_eigh.py,
        # profiles/als_first_iteration_r4.json)
        Gd = G.detach().to(device="cpu", dtype=torch.float64)
        ev, V = torch.linalg.eigh(0.5 * (Gd + Gd.T))
        eig = ev.clamp_min(0.0).float().to(F.device).contiguous()
        Q = V.float().to(F.device).contiguous()
        comm = self.comm if shared else None
        if comm is not None and comm.world_size > 1:          # rank 0's basis on every rank
            R = Q.shape[0]
            both = torch.cat([eig.reshape(1, R), Q]).contiguous()
            comm.broadcast(both, src=0)
            eig, Q = both[0].contiguous(), both[1:].contiguous()
        FQ = rotated_table(F, Q) if need_fq else None
        self.key = (weakref.ref(F), weakref.ref(G), key)
        self.val = (eig, Q, FQ)
        return self.val

    def clear(self):
        self.key = self.val = None
        self.comm = None


EIG_CACHE = _EigCache()


def rotated_table(F: torch.Tensor, Q: torch.Tensor) -> torch.Tensor:
    """F Q for the Woodbury gathers.  On the GPU: the x = Q y rotation kernel (matrix cores at
    rank 128) over every row of F with Q in the place of Q^T (row f -> Q^T f = (f Q)^T),
    written to a new table -- no GEMM library call (hipBLASLt's first call in a process costs
    ~160 ms of the first ALS iteration, profiles/als_first_iteration_r4.json); elsewhere
    torch.mm."""
    R = F.shape[1]
    if not (F.is_cuda and F.dtype == torch.float32 and F.is_contiguous() and R in EXACT_RANKS
            and F.shape[0] < (1 << 31)):
        return torch.mm(F, Q)
    FQ = torch.empty_like(F)
    n = F.shape[0]
    if n:
        rows = torch.arange(n, dtype=torch.int32, device=F.device)
        lib = N.kernels()
        grid = max(1, min(N.num_cus(F.device) * 2, -(-n // 32)))
        N.check(lib.o3s_als_rotate_to(R, Q.contiguous().data_ptr(), rows.data_ptr(), n, F.data_ptr(),
                                      FQ.data_ptr(), grid, N.stream_of(FQ)), "als_rotate(F Q)")
    return FQ


def exact_solve(indptr, cols, w, b, F, G, lam, implicit: bool, out: torch.Tensor, row_range=None,
                eig_basis: bool = False) -> torch.Tensor:
    """Exact per-row solves (csrc/als_exact.hip) written into ``out`` (rows of this CSR,
    or rows [a, b) of it).  Rows with <= 32 ratings and lam_u > 0 take the Woodbury kernel
    (an n x n Cholesky against the eigendecomposition G = Q diag(e) Q^T, gathering rows of
    the rotated table F Q; x = Q y afterwards by als_rotate_kernel), the others the dense
    kernel (register-tile Gram + blocked Cholesky).  G = Y^T Y (implicit only).

    ``eig_basis`` (implicit, compiled ranks): every row is returned in the eigenbasis Q of
    G, y = Q^T x -- the Woodbury rows skip the x = Q y rotation and the dense rows solve the
    rotated system (F Q, diag(eig)) -- so a fit that keeps its tables in that basis
    (models/als.py fit_als) never rotates the large side's table; Q is EIG_CACHE's."""
    dev = F.device
    R = F.shape[1]
    if R not in EXACT_RANKS:
        # zero columns for the padded dimensions: the padded system is block diagonal with
        # a lam_u * I block (implicit: G padded with zeros), so its solution is [x_u, 0]
        Rp = _padded_rank(R)
        Fp = PAD_CACHE.get(F, Rp)
        Gp = None
        if G is not None:
            Gp = torch.zeros((Rp, Rp), dtype=G.dtype, device=G.device)
            Gp[:R, :R] = G
        a0, e0 = (0, indptr.numel() - 1) if row_range is None else row_range
        outp = torch.zeros((e0 - a0, Rp), dtype=torch.float32, device=dev)
        sub = indptr[a0:e0 + 1]
        exact_solve(sub - sub[0] if a0 else sub, cols[int(sub[0]):int(sub[-1])] if a0 else cols,
                    w[int(sub[0]):int(sub[-1])] if a0 else w, b[int(sub[0]):int(sub[-1])] if a0 else b,
                    Fp, Gp, lam[a0:e0].contiguous(), implicit, outp)
        out[a0:e0] = outp[:, :R]
        return out
    n_all = indptr.numel() - 1
    a, e = (0, n_all) if row_range is None else row_range
    cnt = (indptr[a + 1:e + 1] - indptr[a:e])
    small_m = (cnt <= N.kernels().o3s_als_exact_max_small()) & (lam[a:e] > 0)
    idx = torch.arange(a, e, device=dev, dtype=torch.int32)
    small = idx[small_m].contiguous()
    dense = idx[~small_m].contiguous()
    ns, nd = int(small.numel()), int(dense.numel())
    lib = N.kernels()
    st = N.stream_of(out)
    eig_basis = bool(eig_basis and implicit)
    if eig_basis:                        # every rank calls this (shared basis, see _EigCache)
        with trace("als.eig_rotated_table"):
            eig, Q, P = EIG_CACHE.get(F, G, True, shared=True)
    if ns:
        if eig_basis:
            pass
        elif implicit:
            with trace("als.eig_rotated_table"):
                eig, Q, P = EIG_CACHE.get(F, G, True)
        else:
            eig, Q, P = torch.zeros(R, dtype=torch.float32, device=dev), None, F
        with trace("als.woodbury", rows=ns):
            cs = cnt[small_m]
            for kn, m_ in ((16, cs <= 16), (24, (cs > 16) & (cs <= 24)), (32, cs > 24)):
                lst = small[m_].contiguous()
                if lst.numel():
                    N.check(lib.o3s_als_wood_kn(R, kn, indptr.data_ptr(), cols.data_ptr(), w.data_ptr(),
                                                b.data_ptr(), P.data_ptr(), eig.data_ptr(), lam.data_ptr(),
                                                lst.data_ptr(), lst.numel(), out.data_ptr(), st), "als_wood")
        if implicit and not eig_basis:        # x = Q y for the Woodbury rows (als_rotate_kernel)
            with trace("als.rotate", rows=ns):
                QT = Q.T.contiguous()
                grid = max(1, min(N.num_cus(dev) * 2, -(-ns // 32)))
                N.check(lib.o3s_als_rotate(R, QT.data_ptr(), small.data_ptr(), ns, out.data_ptr(), grid, st),
                        "als_rotate")
    if nd:
        with trace("als.dense", rows=nd):
            gd = None
            if eig_basis:                     # the rotated system: F Q and diag(eig)
                F = P
                if DENSE_GDIAG:
                    gd, Gf = eig.float().contiguous(), None
                else:
                    Gf = torch.diag(eig).contiguous()
            else:
                Gf = G.float().contiguous() if implicit else None
            # longest rows first: the waves take rows round robin, so the long tail of
            # popular items spreads over the whole chip instead of finishing last
            order = torch.argsort(cnt[dense - a], descending=True)
            dense_wave(implicit, indptr, cols, w, b, F, Gf, lam, dense[order], out, gdiag=gd)
    return out


def dense_meta(indptr, rows, lam):
    """The dense kernel's per-row metadata, int32 [n][8] in list order:
    {p0 lo, p0 hi, n, u, lam_u bits, 0, 0, 0} (csrc/als_dense.hip DMAs it ahead of use)."""
    rows = rows.long()
    p0 = indptr[rows]
    meta = torch.zeros((rows.numel(), 8), dtype=torch.int32, device=rows.device)
    meta[:, 0:2] = p0.view(torch.int32).view(-1, 2)
    meta[:, 2] = (indptr[rows + 1] - p0).to(torch.int32)
    meta[:, 3] = rows.to(torch.int32)
    meta[:, 4] = lam[rows].float().view(torch.int32)
    return meta


def dense_wave(implicit, indptr, cols, w, b, F, Gf, lam, rows, out, grid=None, gdiag=None):
    """o3s_als_dense_wave over the listed rows (in list order: the caller sorts them longest
    first); rows without ratings are solved here (x = 0: the right-hand side is 0), so every
    row the kernel walks has at least one 16-rating step.  ``gdiag`` (fp32 [R], the
    eigenbasis solves): G = diag(gdiag) instead of ``Gf`` -- the build without the G image
    in LDS (``o3s_als_dense_wave_gd``)."""
    R = F.shape[1]
    cnt = indptr[rows.long() + 1] - indptr[rows.long()]
    empty = cnt == 0
    if bool(empty.any()):
        out[rows[empty].long()] = 0
        rows = rows[~empty]
    n = int(rows.numel())
    if not n:
        return out
    meta = dense_meta(indptr, rows, lam)
    lib = N.kernels()
    if gdiag is not None:
        N.check(lib.o3s_als_dense_wave_gd(R, meta.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                          F.data_ptr(), gdiag.data_ptr(), n, out.data_ptr(),
                                          N.num_cus(F.device) if grid is None else grid, N.stream_of(out)),
                "als_dense_wave_gd")
        return out
    N.check(lib.o3s_als_dense_wave(int(implicit), R, meta.data_ptr(), cols.data_ptr(), w.data_ptr(), b.data_ptr(),
                                   F.data_ptr(), N.ptr(Gf), n, out.data_ptr(),
                                   N.num_cus(F.device) if grid is None else grid, N.stream_of(out)),
            "als_dense_wave")
    return out


def exact_solve_torch(indptr, cols, w, b, F, G, lam, out, row_range=None, chunk_rows: int = 4096):
    """fp64 reference of :func:`exact_solve` (also the CPU path): forms each row's
    A_u = G + sum w y y^T + lam_u I and solves it, in bounded row chunks."""
    dev = F.device
    R = F.shape[1]
    n_all = indptr.numel() - 1
    a0, e0 = (0, n_all) if row_range is None else row_range
    eye = torch.eye(R, dtype=torch.float64, device=dev)
    for a in range(a0, e0, chunk_rows):
        e = min(e0, a + chunk_rows)
        lo, hi = int(indptr[a]), int(indptr[e])
        m = e - a
        rows = torch.repeat_interleave(torch.arange(m, device=dev), indptr[a + 1:e + 1] - indptr[a:e])
        M = torch.zeros((m, R, R), dtype=torch.float64, device=dev)
        rhs = torch.zeros((m, R), dtype=torch.float64, device=dev)
        step = max(1, (1 << 25) // (R * R))          # bounded outer-product temporaries
        for s0 in range(lo, hi, step):
            s1 = min(hi, s0 + step)
            Fg = F[cols[s0:s1].long()].to(torch.float64)
            rr = rows[s0 - lo:s1 - lo]
            M.index_add_(0, rr, Fg[:, :, None] * Fg[:, None, :] * w[s0:s1].to(torch.float64)[:, None, None])
            rhs.index_add_(0, rr, Fg * b[s0:s1].to(torch.float64)[:, None])
        if G is not None:
            M = M + G.to(torch.float64)[None]
        M = M + lam[a:e].to(torch.float64)[:, None, None] * eye[None] + 1e-12 * eye[None]
        out[a:e] = torch.linalg.solve(M, rhs[:, :, None]).squeeze(-1).to(out.dtype)
    return out
