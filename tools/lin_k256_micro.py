"""K = 256 bf16 linears on few output tiles (the d_model-256 projections: M 2048 / 6400 x N 256):
gemm_kernel's double-buffered K loop (RETR_TUNE_LIN_K256 = 1) vs every K-step fetched at once
(2, gemm2.hpp gemm_short_kernel).  Each variant must give the same bytes; 20 calls in a hipGraph,
best of 5 replays.

    python tools/lin_k256_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402
from tools.conv_micro import timeit  # noqa: E402

KNOB = 33
SHAPES = [(2048, 256, 256), (6400, 256, 256), (2048, 512, 256), (2048, 64, 256)]


def main():
    bf = torch.bfloat16
    torch.manual_seed(0)
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        b = torch.randn(N, device="cuda")
        res = torch.randn(M, N, device="cuda")
        dy = torch.randn(M, N, device="cuda").to(bf)
        gate = torch.randn(M, K, device="cuda").to(bf)
        add = torch.randn(M, K, device="cuda").to(bf)
        cases = {
            "fwd f32 +res+drop": lambda y: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b),
                                                 ptr(y), N, 1, M, N, K, 0, ptr(res), N, 0.1, 7,
                                                 stream()),
            "fwd bf16 relu": lambda y: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b),
                                            ptr(y), N, 0, M, N, K, 1, None, 0, 0.0, 0, stream()),
            "dgrad gate+add": lambda y: call("retr_linear_dgrad", 1, ptr(dy), N, ptr(w), K, ptr(y),
                                             K, 0, M, N, K, ptr(add), 0, K, ptr(gate), K, 0,
                                             stream()),
        }
        for name, fn in cases.items():
            f32 = name.startswith("fwd f32")
            cols = K if name.startswith("dgrad") else N
            outs, times = [], []
            for v in (1, 2):
                load().retr_tune(KNOB, v)
                y = torch.zeros(M, cols, device="cuda", dtype=torch.float32 if f32 else bf)
                fn(y)
                torch.cuda.synchronize()
                outs.append(y.clone())
                times.append(timeit(lambda: fn(y)))
            load().retr_tune(KNOB, 0)
            same = "bitwise" if torch.equal(outs[0], outs[1]) else \
                f"DIFF {(outs[0].float() - outs[1].float()).abs().max().item():.3g}"
            print(f"M{M} N{N} K{K} {name:18s} loop {times[0]:6.2f} us  short {times[1]:6.2f} us  "
                  f"{same}", flush=True)


if __name__ == "__main__":
    main()
