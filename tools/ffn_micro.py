"""Device time of the fused FFN kernels (csrc/ffn.hip) against the two-launch path at the cfg2
shapes (d_model 256, F 2048; encoder M 6400, decoder M 2048), per F-split count: 20 calls in a
hipGraph, best of 5.

    python tools/ffn_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import call, load, ptr, stream  # noqa: E402
from tools.conv_micro import timeit  # noqa: E402


def pmc_loop(which, s, n):
    """Eager launches of one fused kernel (encoder shape) for rocprofv3 --pmc passes."""
    bf = torch.bfloat16
    M, C, F = 6400, 256, 2048
    a = torch.randn(M, C, device="cuda").to(bf)
    w1 = (torch.randn(F, C, device="cuda") * 0.05).to(bf)
    w2 = (torch.randn(C, F, device="cuda") * 0.05).to(bf)
    b1, b2 = torch.randn(F, device="cuda"), torch.randn(C, device="cuda")
    x = torch.randn(M, C, device="cuda")
    h = torch.randn(M, F, device="cuda").to(bf)
    y = torch.empty(M, C, device="cuda")
    dh = torch.empty(M, F, device="cuda", dtype=bf)
    dn = torch.empty(M, C, device="cuda", dtype=bf)
    ws = torch.empty(s, M, C, device="cuda")
    for _ in range(n):
        if which == "fwd":
            call("retr_ffn_fwd", ptr(a), C, ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(h), F, ptr(x),
                 C, ptr(y), C, M, C, F, 0.1, 5, ptr(ws), s, stream())
        else:
            call("retr_ffn_bwd_data", ptr(a), C, ptr(w2), ptr(h), F, ptr(w1), ptr(dh), F, ptr(dn),
                 C, M, C, F, ptr(ws), s, stream())
    torch.cuda.synchronize()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "pmc":
        return pmc_loop(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    bf = torch.bfloat16
    C, F = 256, 2048
    for M in (6400, 2048):
        n = torch.randn(M, C, device="cuda").to(bf)
        w1 = (torch.randn(F, C, device="cuda") * 0.05).to(bf)
        w2 = (torch.randn(C, F, device="cuda") * 0.05).to(bf)
        b1 = torch.randn(F, device="cuda")
        b2 = torch.randn(C, device="cuda")
        x = torch.randn(M, C, device="cuda")
        h = torch.empty(M, F, device="cuda", dtype=bf)
        y = torch.empty(M, C, device="cuda")
        dh = torch.empty(M, F, device="cuda", dtype=bf)
        dn = torch.empty(M, C, device="cuda", dtype=bf)
        fl = 2 * 2 * M * C * F
        s0 = int(load().retr_ffn_splits(M, C, F))

        def unfused_fwd():
            ops.k_linear_fwd(n, w1, b1, h, relu=1)
            ops.k_linear_fwd(h, w2, b2, y, res=x, drop_p=0.1, seed=5)

        def unfused_bwd():
            ops.k_linear_dgrad(n, ops._TView(w2), dh, gate=h)
            ops.k_linear_dgrad(dh, ops._TView(w1), dn)
        tu, tub = timeit(unfused_fwd), timeit(unfused_bwd)
        line = (f"M{M} C{C} F{F}: unfused fwd {tu:6.1f} us {fl / tu / 1e6:4.0f} TF | "
                f"bwd {tub:6.1f} us {fl / tub / 1e6:4.0f} TF")
        for s in sorted({1, 2, 4, 8, 16, s0}):
            if (F // 64) % s:
                continue
            ws = torch.empty(s, M, C, device="cuda")
            tf = timeit(lambda: call("retr_ffn_fwd", ptr(n), C, ptr(w1), ptr(b1), ptr(w2),
                                     ptr(b2), ptr(h), F, ptr(x), C, ptr(y), C, M, C, F, 0.1, 5,
                                     ptr(ws), s, stream()))
            tb = timeit(lambda: call("retr_ffn_bwd_data", ptr(n), C, ptr(w2), ptr(h), F, ptr(w1),
                                     ptr(dh), F, ptr(dn), C, M, C, F, ptr(ws), s, stream()))
            line += (f" | fused s{s}{'*' if s == s0 else ''} fwd {tf:6.1f} bwd {tb:6.1f} us")
        print(line, flush=True)


if __name__ == "__main__":
    main()
