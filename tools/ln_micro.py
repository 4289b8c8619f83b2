"""Device time of the fused LayerNorm backward (retr_layernorm_bwd2: dy + dy2 bf16, fp32 x /
addend, fp32 dx, bf16 dropout(dx), parameter partial rows left to the caller) at the cfg2 shapes
per launch shape (retr_tune RETR_TUNE_LN_BWD = 27): 20 calls in a hipGraph, best of 5 replays.

    python tools/ln_micro.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402
from tools.conv_micro import timeit  # noqa: E402


def main():
    bf = torch.bfloat16
    C = 256
    for M in (6400, 2048):
        dy = torch.randn(M, C, device="cuda").to(bf)
        dy2 = torch.randn(M, C, device="cuda").to(bf)
        x = torch.randn(M, C, device="cuda")
        add = torch.randn(M, C, device="cuda")
        g = torch.randn(C, device="cuda")
        mean = torch.randn(M, device="cuda")
        rstd = torch.rand(M, device="cuda") + 0.5
        dx = torch.empty(M, C, device="cuda")
        dxd = torch.empty(M, C, device="cuda", dtype=bf)
        ws = torch.empty(int(load().retr_layernorm_bwd_workspace(M, C)) // 4, device="cuda")
        npar = ctypes.c_int(0)
        out = []
        for cfg in (0, 1, 2, 3, 4, 5, 6):
            load().retr_tune(27, cfg)
            t = timeit(lambda: call("retr_layernorm_bwd2", 1, ptr(dy), ptr(dy2), C, ptr(x), C,
                                    ptr(g), ptr(mean), ptr(rstd), M, C, ptr(dx), C, ptr(add),
                                    None, None, ptr(ws), ptr(dxd), C, 0.1, 7,
                                    ctypes.addressof(npar), stream()))
            out.append(f"c{cfg}: {t:6.2f}us")
        load().retr_tune(27, 0)
        print(f"ln_bwd2 M{M} C{C} | " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
