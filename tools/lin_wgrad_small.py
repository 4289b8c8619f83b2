"""Ungrouped bf16 linear weight gradients below the LDS-DMA size rule (N < 512): the register-
staged 64x64 kernel (knob 11 = 0) vs the LDS-DMA tiles (11 = 5 / 6 / 7) over split counts
(knob 17), with the bias gradient and accumulate = 1 as in the step; 20 calls in a hipGraph.

    python tools/lin_wgrad_small.py
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
    lib = load()
    for M, N, K in ((6400, 256, 2048), (2048, 512, 256), (2048, 512, 512), (2048, 256, 2048)):
        dy = torch.randn(M, N, device="cuda").to(bf)
        x = torch.randn(M, K, device="cuda").to(bf)
        dw = torch.zeros(N, K, device="cuda")
        db = torch.zeros(N, device="cuda")
        ref = ref_b = None
        print(f"wgrad M{M} N{N} K{K}:", flush=True)
        for v in (0, 5, 6, 7):
            for s in (0, 2, 4, 8, 16, 32):
                lib.retr_tune(11, v)
                lib.retr_tune(17, s)
                dw.zero_()
                db.zero_()
                ops.k_linear_wgrad(dy, x, dw, db)
                torch.cuda.synchronize()
                if ref is None:
                    ref, ref_b = dw.clone(), db.clone()
                err = ((dw - ref).norm() / ref.norm()).item()
                errb = ((db - ref_b).norm() / ref_b.norm()).item()
                t = timeit(lambda: ops.k_linear_wgrad(dy, x, dw, db))
                print(f"   v{v} s{s:2d} {t:6.1f} us {2 * M * N * K / t / 1e6:5.0f} TF "
                      f"err {err:.1e} {errb:.1e}", flush=True)
        lib.retr_tune(11, 0)
        lib.retr_tune(17, 0)


if __name__ == "__main__":
    main()
