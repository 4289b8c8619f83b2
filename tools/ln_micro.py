"""Device time of the row-wise memory-bound kernels of the transformer step (LayerNorm forward /
backward with its parameter reduction, dropout mask application) at the cfg2 shapes
(encoder 6400 x 256 rows, decoder 2048 x 256), 20 calls in a hipGraph, best of 5 replays,
with the achieved bandwidth on the algorithmic bytes.

    python tools/ln_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import call, ptr  # noqa: E402

DEV = "cuda"


def timeit(fn, n=20):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(n):
            fn()
    best = float("inf")
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def main():
    bf = torch.bfloat16
    C = 256
    for M in (6400, 2048):
        x = torch.randn(M, C, device=DEV)
        gamma, beta = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
        pos = torch.randn(400, C, device=DEV)
        y, y2 = (torch.empty(M, C, dtype=bf, device=DEV) for _ in range(2))
        mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
        fwd = lambda: call("retr_layernorm_fwd", 1, ptr(x), C, ptr(gamma), ptr(beta), 1e-5, M, C,  # noqa: E731
                           ptr(y), C, ptr(y2), ptr(pos), 400, ptr(mean), ptr(rstd), ops._st())
        t = timeit(fwd)
        nb = M * C * (4 + 2 + 2)
        print(f"ln_fwd   M{M}: {t:6.2f} us  {nb / t / 1e3:6.0f} GB/s", flush=True)
        dy, dy2 = torch.randn(M, C, device=DEV).to(bf), torch.randn(M, C, device=DEV).to(bf)
        add = torch.randn(M, C, device=DEV)
        dx = torch.empty(M, C, device=DEV)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        ws = ops.ln_workspace(M, C, x.device)
        bwd = lambda: call("retr_layernorm_bwd", 1, ptr(dy), ptr(dy2), C, ptr(x), C, ptr(gamma),  # noqa: E731
                           ptr(mean), ptr(rstd), M, C, ptr(dx), C, ptr(add), ptr(dg), ptr(db),
                           ptr(ws), ops._st())
        t = timeit(bwd)
        nb = M * C * (2 + 2 + 4 + 4 + 4)
        print(f"ln_bwd   M{M}: {t:6.2f} us  {nb / t / 1e3:6.0f} GB/s (incl. param reduce)",
              flush=True)
        ydrop = torch.empty(M, C, dtype=bf, device=DEV)
        dr = lambda: ops.k_dropout_apply(x, ydrop, 0.1, 99)  # noqa: E731
        t = timeit(dr)
        nb = M * C * (4 + 2)
        print(f"dropout  M{M}: {t:6.2f} us  {nb / t / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
