"""Device time of the bf16 linear weight gradient (retr_linear_wgrad) on the cfg2 vocabulary
head (dW[30522][512] += dY^T X over 2048 tokens, with the bias gradient) per RETR_TUNE_LIN_WGRAD
variant; 20 calls in a hipGraph, best of 5 replays.

    python tools/wgrad_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import load  # noqa: E402
from tools.conv_micro import timeit  # noqa: E402


def main():
    bf = torch.bfloat16
    for M, N, K in ((2048, 30528, 512), (2048, 512, 512), (6400, 256, 2048)):
        dy = torch.randn(M, N, device="cuda").to(bf)
        x = torch.randn(M, K, device="cuda").to(bf)
        dw = torch.zeros(N, K, device="cuda")
        db = torch.zeros(N, device="cuda")
        ref = None
        line = f"wgrad M{M} N{N} K{K}:"
        for v in (1, 0, 2, 4):
            load().retr_tune(11, v)
            dw.zero_()
            db.zero_()
            ops.k_linear_wgrad(dy, x, dw, db)
            torch.cuda.synchronize()
            err = 0.0 if ref is None else ((dw - ref).norm() / ref.norm()).item()
            ref = dw.clone() if ref is None else ref
            t = timeit(lambda: ops.k_linear_wgrad(dy, x, dw, db))
            line += f"  v{v} {t:6.1f} us {2 * M * N * K / t / 1e6:5.0f} TF err {err:.1e}"
        load().retr_tune(11, 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
