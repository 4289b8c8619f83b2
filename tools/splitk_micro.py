"""Device-time sweep of the split-K slice count for the long-reduction linears of cfg2 (FFN
down-projections, FFN up-projection data gradients, the vocabulary head's data gradient):
retr_linear_fwd_splitk / retr_linear_dgrad_splitk at splits 1..8 vs the single-pass kernel.
20 calls captured in a hipGraph, best of 5 replays.

    python tools/splitk_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402

DEV = "cuda"
# (kind, M, N_out, K_reduction, residual/gate)
SHAPES = [("fwd", 6400, 256, 2048, 1), ("fwd", 2048, 256, 2048, 1), ("fwd", 6400, 256, 2048, 0),
          ("dgrad", 6400, 256, 2048, 0), ("dgrad", 2048, 256, 2048, 0),
          ("dgrad", 2048, 512, 30528, 1)]


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
    for kind, M, N, K, extra in SHAPES:
        out = []
        ws = torch.empty(8 * M * N, device=DEV)
        if kind == "fwd":
            x = torch.randn(M, K, device=DEV).to(bf)
            w = (torch.randn(N, K, device=DEV) * 0.02).to(bf)
            b = torch.randn(N, device=DEV)
            res = torch.randn(M, N, device=DEV) if extra else None
            y = torch.empty(M, N, device=DEV)
            single = lambda: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N, 1,  # noqa: E731
                                  M, N, K, 0, ptr(res), N, 0.1, 5, stream())
            split = lambda s: call("retr_linear_fwd_splitk", 1, ptr(x), K, ptr(w), K, ptr(b),  # noqa: E731
                                   ptr(y), N, 1, M, N, K, 0, ptr(res), N, 0.1, 5, ptr(ws), s,
                                   stream())
        else:
            dy = torch.randn(M, K, device=DEV).to(bf)
            w = (torch.randn(K, N, device=DEV) * 0.02).to(bf)      # W [K_red][N_out] row-major
            gate = torch.randn(M, N, device=DEV).to(bf) if extra else None
            dx = torch.empty(M, N, dtype=bf, device=DEV)
            single = lambda: call("retr_linear_dgrad", 1, ptr(dy), K, ptr(w), N, ptr(dx), N, 0,  # noqa: E731
                                  M, K, N, None, 0, 0, ptr(gate), N, 0, stream())
            split = lambda s: call("retr_linear_dgrad_splitk", 1, ptr(dy), K, ptr(w), N, ptr(dx),  # noqa: E731
                                   N, 0, M, K, N, None, 0, 0, ptr(gate), N, 0, ptr(ws), s,
                                   stream())
        fl = 2.0 * M * N * K
        t = timeit(single)
        out.append(f"1:{t:6.1f}us {fl / t / 1e6:4.0f}TF")
        for s in (2, 3, 4, 5, 6, 8):
            t = timeit(lambda: split(s))
            out.append(f"{s}:{t:6.1f}us {fl / t / 1e6:4.0f}TF")
        plan = load().retr_linear_splits(1, M, N, K)
        print(f"{kind:5s} M{M} N{N} K{K} x{extra} plan{plan} | " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
