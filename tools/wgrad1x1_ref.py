"""1x1 convolution weight gradients: retr_conv2d_wgrad (split-K fp32 slabs, the kernel alone)
vs hipBLASLt's dy^T x (torch.mm, bf16 out) on the cfg2 1x1 shapes.  Eager, 20 calls, best of 3.

    python tools/wgrad1x1_ref.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import call, load, ptr  # noqa: E402

SHAPES = [  # (N, H, Ci, Co)
    (16, 40, 256, 1024), (16, 80, 128, 512), (16, 40, 1024, 256), (16, 80, 512, 128),
    (16, 20, 512, 2048), (16, 160, 256, 128), (16, 20, 2048, 512), (16, 160, 64, 256),
]


def timeit(fn, n=20):
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def main():
    bf = torch.bfloat16
    lib = load()
    tiles = [int(t) for t in os.environ.get("RETR_WTILES", "0").split(",")]
    for N, H, Ci, Co in SHAPES:
        P = N * H * H
        x = torch.randn(P, Ci, device="cuda").to(bf)
        dy = torch.randn(P, Co, device="cuda").to(bf)
        fl = 2.0 * P * Ci * Co
        line = f"P{P} Co{Co} Ci{Ci}:"
        for t in tiles:
            lib.retr_tune(9, t)
            s = lib.retr_conv2d_wgrad_splits(1, N, H, H, Ci, Co, 1, 1, 1, 0, 1)
            ws = torch.empty(s, Co, Ci, device="cuda")
            f = lambda: call("retr_conv2d_wgrad", 1, ptr(dy), ptr(x), N, H, H, Ci, ptr(ws), Co,  # noqa: E731
                             1, 1, 1, 0, 1, ops._st())
            f()
            us = timeit(f)
            line += f" retr[t{t} s{s}] {us:6.1f} us {fl / us / 1e6:4.0f} TF |"
        lib.retr_tune(9, 0)
        dyt = dy.t()
        us = timeit(lambda: torch.mm(dyt, x))
        line += f" hipBLASLt {us:6.1f} us {fl / us / 1e6:4.0f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
