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


def main():
    bf = torch.bfloat16
    for M, N, K, relu, f32 in SHAPES:
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=torch.float32 if f32 else bf)
        out = []
        for tile in (0, 1, 2, 3, 4, 6, 8, 9):
            load().retr_tune(6, tile)
            t = timeit(lambda: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N,
                                    f32, M, N, K, relu, None, 0, 0.0, 0, stream()))
            out.append(f"t{tile}: {t:6.1f}us {2 * M * N * K / t / 1e6:4.0f}TF")
        load().retr_tune(6, 0)
        print(f"fwd M{M} N{N} K{K} | " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
