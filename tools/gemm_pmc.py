"""Eager loop of one convolution GEMM shape for rocprofv3 --pmc passes (per-dispatch counters of
the implicit-GEMM kernel: wave states, LDS traffic / bank conflicts, instruction mix).

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... -- python tools/gemm_pmc.py fwd3 [tile] [n]

shapes: fwd3 = 3x3 conv 40x40x256 -> 256 (M 25600, N 256, K 2304), fwd1 = 1x1 conv
80x80x128 -> 512, gemm = the plain GEMM of fwd3's size (retr_linear_fwd), ffn = the encoder FFN
expansion (M 6400, N 2048, K 256, bias + ReLU).  tile: the
RETR_TUNE_BIG_TILE override (0 = built-in choice).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402

BF = 1


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "fwd3"
    tile = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    bf = torch.bfloat16
    load().retr_tune(6, tile)
    if shape in ("gemm", "ffn"):
        M, N, K = (25600, 256, 2304) if shape == "gemm" else (6400, 2048, 256)
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=bf)
        fl = 2.0 * M * N * K
        relu = int(shape == "ffn")
        fn = lambda: call("retr_linear_fwd", BF, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N, 0,  # noqa: E731
                          M, N, K, relu, None, 0, 0.0, 0, stream())
    elif shape == "dg1":   # 1x1 data gradient 80x80x512 <- 128 with the residual addend
        Nb, H, C, Co = 16, 80, 512, 128
        dy = torch.randn(Nb * H * H * Co, device="cuda").to(bf)
        w = (torch.randn(Co * C, device="cuda") * 0.05).to(bf)
        add = torch.randn(Nb * H * H * C, device="cuda").to(bf)
        dx = torch.empty(Nb * H * H * C, dtype=bf, device="cuda")
        fl = 2.0 * Nb * H * H * Co * C
        fn = lambda: call("retr_conv2d_dgrad", BF, ptr(dy), Nb, H, H, C, ptr(w), ptr(dx), Co,  # noqa: E731
                          1, 1, 1, 0, 1, ptr(add), None, stream())
    else:
        Nb, H, C, Co, k, p = (16, 40, 256, 256, 3, 1) if shape == "fwd3" else (16, 80, 128, 512, 1, 0)
        x = torch.randn(Nb * H * H * C, device="cuda").to(bf)
        w = (torch.randn(Co * k * k * C, device="cuda") * 0.05).to(bf)
        b = torch.randn(Co, device="cuda")
        y = torch.empty(Nb * H * H * Co, dtype=bf, device="cuda")
        fl = 2.0 * Nb * H * H * Co * k * k * C
        res = torch.randn(Nb * H * H * Co, device="cuda").to(bf) if shape == "fwd1" else None
        fn = lambda: call("retr_conv2d_fwd", BF, ptr(x), Nb, H, H, C, ptr(w), ptr(b), ptr(res),  # noqa: E731
                          ptr(y), Co, k, k, 1, p, 1, 1, stream())
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    print(f"{shape} tile {tile}: {us:.1f} us/call (eager, incl. launch gaps) "
          f"{fl / us / 1e6:.0f} TF/s", flush=True)
    load().retr_tune(6, 0)


if __name__ == "__main__":
    main()
