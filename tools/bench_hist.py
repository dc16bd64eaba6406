"""Micro-benchmark of the tree histogram kernel: sequential vs random row order, 1 vs
256 node segments (62.5M x 64 uint8 bins, 32 bins, regression stats)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orange3_spark_amd.ops import trees as T  # noqa: E402

n, F, B = int(sys.argv[1]) if len(sys.argv) > 1 else 62_500_000, 64, 32
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
bins = torch.randint(0, B, (n, F), device=dev, dtype=torch.uint8, generator=g)
y = torch.randn(n, device=dev, generator=g)
res = {}
for name, order in (("seq", torch.arange(n, device=dev, dtype=torch.int32)),
                    ("rand", torch.randperm(n, device=dev, generator=g).to(torch.int32))):
    for nseg in (1, 256):
        cuts = torch.linspace(0, n, nseg + 1, device=dev).long()
        lo, hi = cuts[:-1].contiguous(), cuts[1:].contiguous()
        node = torch.arange(nseg, device=dev)
        for chunk in (1 << 13, 1 << 15):
            yp = y[order.long()].contiguous()          # position-ordered labels (the GBT path)
            T.node_hist(bins, order, yp, None, lo, hi, node, nseg, B, 3, False, chunk=chunk, ypos=True)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                T.node_hist(bins, order, yp, None, lo, hi, node, nseg, B, 3, False, chunk=chunk, ypos=True)
            torch.cuda.synchronize()
            res[f"{name}_seg{nseg}_chunk{chunk}"] = round((time.perf_counter() - t) / 3 * 1e3, 3)
print(json.dumps({"n": n, "F": F, "B": B, "ms": res}))
