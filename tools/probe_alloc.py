"""First-touch cost of fresh device memory: times torch.empty (hipMalloc through the
caching allocator) and the first vs second fill of 1/2/8/32 GB blocks in a fresh process,
then the same sizes served from the allocator's cache."""
import json
import time

import torch


def t(fn):
    torch.cuda.synchronize()
    a = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, time.perf_counter() - a


def main():
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    out = []
    for gb in (1, 2, 8, 32):
        n = gb << 28
        x, ta = t(lambda: torch.empty(n, dtype=torch.float32, device=dev))
        _, t1 = t(lambda: x.fill_(1.0))
        _, t2 = t(lambda: x.fill_(2.0))
        del x
        y, tc = t(lambda: torch.empty(n, dtype=torch.float32, device=dev))
        _, t3 = t(lambda: y.fill_(3.0))
        del y
        out.append({"GB": gb, "empty_fresh_ms": round(ta * 1e3, 2), "first_fill_ms": round(t1 * 1e3, 2),
                    "second_fill_ms": round(t2 * 1e3, 2), "empty_cached_ms": round(tc * 1e3, 3),
                    "fill_cached_ms": round(t3 * 1e3, 2)})
        print(json.dumps(out[-1]), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
