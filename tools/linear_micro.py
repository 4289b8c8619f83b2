"""Device time of the cfg2 transformer's single (non-grouped) bf16 linear GEMMs per big-GEMM
tile (retr_tune RETR_TUNE_BIG_TILE; shapes routed to launch_big): 20 calls in a hipGraph, best
of 5 replays.

    python tools/linear_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402
from tools.conv_micro import timeit  # noqa: E402

# (M, N, K, relu, y fp32): FFN expansions (encoder / decoder), the vocabulary head
SHAPES = [(6400, 2048, 256, 1, 0), (2048, 2048, 256, 1, 0), (2048, 30528, 512, 0, 1),
          (6400, 512, 256, 0, 0), (2048, 512, 512, 1, 0)]
# the decoder-side (2048 caption tokens) projections of the cfg2 step: (M, N, K, relu, y fp32)
SMALL = [(2048, 256, 256, 0, 0), (2048, 512, 256, 0, 0), (2048, 768, 256, 0, 0),
         (2048, 256, 2048, 0, 0), (6400, 256, 256, 0, 0), (6400, 768, 256, 0, 0)]


def splitk():
    """Long-reduction, few-tile linears (FFN down-projection forward, up-projection data
    gradient): the split-K path (fp32 slabs + ordered epilogue launch) vs single-pass tiles."""
    bf = torch.bfloat16
    for M, N, K in ((2048, 256, 2048), (6400, 256, 2048)):
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        b = torch.randn(N, device="cuda")
        res = torch.randn(M, N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=bf)
        s = int(load().retr_linear_splits(1, M, N, K))
        ws = torch.empty(max(s, 1), M, N, device="cuda")
        out = []
        t = timeit(lambda: call("retr_linear_fwd_splitk", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N,
                                0, M, N, K, 0, ptr(res), N, 0.1, 3, ptr(ws), s, stream()))
        out.append(f"split{s}: {t:6.1f}us")
        for tile in (0, 10, 11, 12, 6):
            load().retr_tune(6, tile)
            t = timeit(lambda: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N, 0,
                                    M, N, K, 0, ptr(res), N, 0.1, 3, stream()))
            out.append(f"t{tile}: {t:6.1f}us")
        load().retr_tune(6, 0)
        print(f"fwd   M{M} N{N} K{K} res+drop | " + " | ".join(out), flush=True)
        # data gradient dX[M][N] = dY[M][K] W[K][N] (W row-major [K][N]: w_trans 0), ReLU gate
        dy = torch.randn(M, K, device="cuda").to(bf)
        wk = (torch.randn(K, N, device="cuda") * 0.05).to(bf)
        gate = torch.randn(M, N, device="cuda").to(bf)
        dx = torch.empty(M, N, device="cuda", dtype=bf)
        s = int(load().retr_linear_splits(1, M, N, K))
        out = []
        t = timeit(lambda: call("retr_linear_dgrad_splitk", 1, ptr(dy), K, ptr(wk), N, ptr(dx), N, 0,
                                M, K, N, None, 0, 0, ptr(gate), N, 0, ptr(ws), s, stream()))
        out.append(f"split{s}: {t:6.1f}us")
        for tile in (0, 10, 11, 12, 6):
            load().retr_tune(6, tile)
            t = timeit(lambda: call("retr_linear_dgrad", 1, ptr(dy), K, ptr(wk), N, ptr(dx), N, 0,
                                    M, K, N, None, 0, 0, ptr(gate), N, 0, stream()))
            out.append(f"t{tile}: {t:6.1f}us")
        load().retr_tune(6, 0)
        print(f"dgrad M{M} N{N} K{K} gate     | " + " | ".join(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "splitk":
        splitk()
        return
    bf = torch.bfloat16
    small = len(sys.argv) > 1 and sys.argv[1] == "small"
    tiles = (0, 2, 4, 5, 6, 8, 9, 10, 11, 12) if small else (0, 1, 2, 3, 4, 6, 8, 9)
    if os.environ.get("RETR_SWEEP_S1"):
        tiles = (0, 13, 14, 15)
    for M, N, K, relu, f32 in (SMALL if small else SHAPES):
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=torch.float32 if f32 else bf)
        out = []
        for tile in tiles:
            load().retr_tune(6, tile)
            t = timeit(lambda: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N,
                                    f32, M, N, K, relu, None, 0, 0.0, 0, stream()))
            out.append(f"t{tile}: {t:6.1f}us {2 * M * N * K / t / 1e6:4.0f}TF")
        load().retr_tune(6, 0)
        print(f"fwd M{M} N{N} K{K} | " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
