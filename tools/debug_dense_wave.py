#!/usr/bin/env python
"""Diagnostic of als_dense_wave_kernel (o3s_als_dense_wave_dbg): decodes the accumulator
tiles dumped after the system is assembled (A) and after the forward factorisation
(U_pi, X_p = L_pp^-1) plus y, and compares each tile with the fp64 reference."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rowof(v, h):
    return (v & 3) + 8 * (v >> 2) + 4 * h


def main():
    from orange3_spark_amd.models import als as AE
    from orange3_spark_amd.ops import _native as N
    from orange3_spark_amd.ops import als as AO
    out = {}
    for R in (64, 128):
        for implicit in (False, True):
            NT = R // 32
            NL = NT * (NT + 1) // 2
            tiles = [(j, i) for j in range(NT) for i in range(j, NT)]
            g = torch.Generator().manual_seed(R)
            n_rows, n_other = 8, 500
            lens = torch.tensor([40, 41, 47, 63, 64, 65, 100, 120])
            indptr = torch.zeros(n_rows + 1, dtype=torch.int64)
            indptr[1:] = torch.cumsum(lens, 0)
            nnz = int(indptr[-1])
            cols = torch.randint(0, n_other, (nnz,), generator=g, dtype=torch.int32)
            vals = torch.randn(nnz, generator=g) * 2
            F = torch.randn((n_other, R), generator=g) / R ** 0.5
            w, b, pos = AE._weights(vals, implicit, 2.0)
            lam = (0.05 * lens.float()).float()
            G = (F.double().T @ F.double()).float() if implicit else None
            dev = "cuda"
            d_ = [x.to(dev) for x in (indptr, cols, w, b, F, lam)]
            Gd = G.to(dev).contiguous() if implicit else None
            rows = torch.arange(n_rows, dtype=torch.int32, device=dev)
            X = torch.zeros((n_rows, R), device=dev)
            dbg = torch.full((128 * NL * 1024 + 64 * R,), float("nan"), device=dev)
            meta = AO.dense_meta(d_[0], rows, d_[5])
            N.check(N.kernels().o3s_als_dense_wave_dbg(int(implicit), R, meta.data_ptr(), d_[1].data_ptr(),
                                                       d_[2].data_ptr(), d_[3].data_ptr(), d_[4].data_ptr(),
                                                       N.ptr(Gd), n_rows, X.data_ptr(), 1, dbg.data_ptr(),
                                                       N.stream_of(X)), "dbg")
            torch.cuda.synchronize()
            D = dbg.cpu().numpy().astype(np.float64)
            res = []
            for r in range(n_rows):
                a, e = int(indptr[r]), int(indptr[r + 1])
                Y = F.double().numpy()[cols[a:e].numpy()]
                A = (Y.T * w[a:e].double().numpy()) @ Y + float(lam[r]) * np.eye(R)
                if implicit:
                    A += G.double().numpy()
                rhs = Y.T @ b[a:e].double().numpy()
                U = np.linalg.cholesky(A).T
                y = np.linalg.solve(U.T, rhs)

                def tile(stage, t):
                    raw = D[((r * 2 + stage) * NL + t) * 1024:((r * 2 + stage) * NL + t + 1) * 1024].reshape(16, 64)
                    M = np.zeros((32, 32))
                    for v in range(16):
                        for l in range(64):
                            M[rowof(v, l >> 5), l & 31] = raw[v, l]
                    return M
                errs = {}
                for t, (j, i) in enumerate(tiles):
                    refA = A[32 * j:32 * j + 32, 32 * i:32 * i + 32]
                    errs[f"A{j}{i}"] = float(np.abs(tile(0, t) - refA).max() / np.abs(refA).max())
                    if i == j:
                        refX = np.linalg.inv(U[32 * j:32 * j + 32, 32 * j:32 * j + 32].T)
                        errs[f"X{j}"] = float(np.abs(tile(1, t) - refX).max() / np.abs(refX).max())
                    else:
                        refU = U[32 * j:32 * j + 32, 32 * i:32 * i + 32]
                        errs[f"U{j}{i}"] = float(np.abs(tile(1, t) - refU).max() / max(np.abs(refU).max(), 1e-30))
                yk = D[128 * NL * 1024 + r * R:128 * NL * 1024 + (r + 1) * R]
                errs["y"] = float(np.abs(yk - y).max() / np.abs(y).max())
                xr = np.linalg.solve(A, rhs)
                errs["x"] = float(np.abs(X[r].cpu().double().numpy() - xr).max() / np.abs(xr).max())
                res.append(errs)
            worst = {k: max(e[k] for e in res) for k in res[0]}
            out[f"R{R}_{'impl' if implicit else 'expl'}"] = worst
            print(R, implicit, json.dumps({k: round(v, 6) for k, v in worst.items()}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
