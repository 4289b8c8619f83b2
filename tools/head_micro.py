"""Device time of the decode step's vocabulary GEMM (M = 64 caption rows, N = 30528 padded
vocabulary, K = 512, bf16 operands, fp32 logits) per big-GEMM tile (retr_tune
RETR_TUNE_BIG_TILE): 20 calls in a hipGraph, best of 5 replays; achieved weight-streaming GB/s.

    python tools/head_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402
from tools.conv_micro import timeit  # noqa: E402


def main():
    bf = torch.bfloat16
    for M, N, K in ((64, 30528, 512), (320, 30528, 512), (64, 512, 512)):
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda")
        out = []
        for tile in tuple(int(t) for t in os.environ.get("HEAD_TILES", "0,1,2,4,6,8,9").split(",")):
            load().retr_tune(6, tile)
            t = timeit(lambda: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N,
                                    1, M, N, K, 0, None, 0, 0.0, 0, stream()))
            out.append(f"t{tile}: {t:6.1f}us {2 * N * K / t / 1e3:5.0f}GB/s")
        load().retr_tune(6, 0)
        print(f"M{M} N{N} K{K} | " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
