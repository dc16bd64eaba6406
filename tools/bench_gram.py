"""X^T X over millions of rows in fp64 on MI355X: plain GEMM vs block-batched GEMM."""
import json
import time

import torch


def t(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / reps * 1e3


def main():
    res = {}
    for n, d in ((4_000_000, 64), (4_000_000, 8), (20_000_000, 256)):
        X = torch.randn((n, d), dtype=torch.float64, device="cuda")
        r = {"plain_ms": t(lambda: X.T @ X)}
        for bs in (1024, 4096, 16384):
            nb = n // bs
            r[f"bmm{bs}_ms"] = t(lambda: torch.bmm(X[: nb * bs].view(nb, bs, d).transpose(1, 2),
                                                   X[: nb * bs].view(nb, bs, d)).sum(0))
        Xf = X.float()
        r["fp32_plain_ms"] = t(lambda: Xf.T @ Xf)
        r["gemv_fp64_ms"] = t(lambda: X.T @ X[:, 0])
        nb = n // 4096
        r["gemv_bmm4096_ms"] = t(lambda: torch.bmm(X[: nb * 4096].view(nb, 4096, d).transpose(1, 2),
                                                   X[: nb * 4096, :1].reshape(nb, 4096, 1)).sum(0))
        r["colsum_ms"] = t(lambda: X.sum(0))
        res[f"{n}x{d}"] = {k: round(v, 3) for k, v in r.items()}
        print(json.dumps(res), flush=True)
        del X, Xf


if __name__ == "__main__":
    main()
