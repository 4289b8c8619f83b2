"""On-GPU sweep of the grouped linear launches (csrc/linear_group.hip) on the cfg2 transformer
shapes: every tile / ring-depth / K-slice override of ``retr_tune`` against the single-GEMM
launches they replace.  Each variant: 20 calls captured into a hipGraph, device time per call (best of 5 replays).

    python tools/group_micro.py > profiles/r2_group_micro.txt
"""
import itertools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import load  # noqa: E402

DEV = "cuda"
G_TILE, G_STAGES, W_TILE, W_STAGES, W_KC = range(5)

FWD = {"enc_attn qk|v": [(6400, 512, 256), (6400, 256, 256)],
       "dec_self qk|v": [(2048, 512, 256), (2048, 256, 256)],
       "dec_cross q|k|v": [(2048, 256, 256), (6400, 256, 256), (6400, 256, 256)]}
WGRAD = {"enc_attn": [(6400, 256, 256), (6400, 512, 256), (6400, 256, 256)],
         "enc_ffn": [(6400, 256, 2048), (6400, 2048, 256)],
         "dec_self": [(2048, 256, 256), (2048, 512, 256), (2048, 256, 256)],
         "dec_cross": [(2048, 256, 256), (2048, 256, 256), (6400, 256, 256), (6400, 256, 256)],
         "dec_ffn": [(2048, 256, 2048), (2048, 2048, 256)]}


def timeit(fn, n=20):
    """Device time per call: n calls captured into one hipGraph (no host launch cost),
    replayed 5 times, best replay."""
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(n):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def tune(knob, v):
    load().retr_tune(knob, v)


def one_wgrad(name, tile, st, kc):
    """A single weight-gradient variant (for rocprofv3 runs: GEMM vs slab-sum split)."""
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(0)
    items = [(torch.randn(M, N, generator=g).to(DEV).to(bf),
              torch.randn(M, K, generator=g).to(DEV).to(bf), torch.zeros(N, K, device=DEV),
              torch.zeros(N, device=DEV), True) for M, N, K in WGRAD[name]]
    tune(W_TILE, tile)
    tune(W_STAGES, st)
    tune(W_KC, kc)
    t = timeit(lambda: ops.k_linear_wgrad_group(items))
    print(f"wgrad {name} {tile} S{st} kc{kc}: {t:.2f} us")


def main():
    if len(sys.argv) > 1:
        return one_wgrad(sys.argv[1], *map(int, sys.argv[2:5]))
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(0)
    rnd = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
    for name, shapes in FWD.items():
        items = []
        for M, N, K in shapes:
            items.append((rnd(M, K).to(bf), (rnd(N, K) * 0.05).to(bf), rnd(N),
                          torch.empty(M, N, dtype=bf, device=DEV)))
        flops = sum(2.0 * M * N * K for M, N, K in shapes)
        t = timeit(lambda: [ops.k_linear_fwd(*it) for it in items])
        print(f"fwd   {name:18s} singles           {t:8.2f} us {flops / t / 1e6:7.1f} TF/s")
        dg = [(rnd(M, N).to(bf), ops._TView((rnd(N, K) * 0.05).to(bf)),
               torch.empty(M, K, dtype=bf, device=DEV)) for M, N, K in
              [(M, N, K) for M, K, N in shapes]]
        td = timeit(lambda: [ops.k_linear_dgrad(*it) for it in dg])
        print(f"dgrad {name:18s} singles           {td:8.2f} us {flops / td / 1e6:7.1f} TF/s")
        for tile, st in [(64, 2), (64, 4), (128, 1), (128, 2), (128, 3)]:
            tune(G_TILE, tile)
            tune(G_STAGES, st)
            t = timeit(lambda: ops.k_linear_fwd_group(items))
            td = timeit(lambda: ops.k_linear_dgrad_group(dg))
            print(f"fwd   {name:18s} group {tile:3d} S{st}      {t:8.2f} us "
                  f"{flops / t / 1e6:7.1f} TF/s   dgrad {td:8.2f} us {flops / td / 1e6:7.1f} TF/s",
                  flush=True)
        tune(G_TILE, 0)
        tune(G_STAGES, 0)
    for name, shapes in WGRAD.items():
        items = []
        for M, N, K in shapes:
            items.append((rnd(M, N).to(bf), rnd(M, K).to(bf), torch.zeros(N, K, device=DEV),
                          torch.zeros(N, device=DEV), True))
        flops = sum(2.0 * M * N * K for M, N, K in shapes)
        t = timeit(lambda: [ops.k_linear_wgrad(*it[:4], accumulate=True) for it in items])
        print(f"wgrad {name:18s} singles           {t:8.2f} us {flops / t / 1e6:7.1f} TF/s")
        for (tile, st), kc in itertools.product([(64, 2), (64, 4), (128, 2), (128, 3)],
                                                [0, 256, 512, 1024, 2048]):
            tune(W_TILE, tile)
            tune(W_STAGES, st)
            tune(W_KC, kc)
            t = timeit(lambda: ops.k_linear_wgrad_group(items))
            print(f"wgrad {name:18s} group {tile:3d} S{st} kc{kc:4d} {t:8.2f} us "
                  f"{flops / t / 1e6:7.1f} TF/s", flush=True)
        for k in (W_TILE, W_STAGES, W_KC):
            tune(k, 0)


if __name__ == "__main__":
    main()
