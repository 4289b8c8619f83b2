"""Device time of an attention out-projection (M x 256 x 256, bias, dropout 0.1, fp32 residual)
followed by the next block's pre-norm LayerNorm (LN(x), LN(x) + pos, mean, rstd): the separate
retr_linear_fwd + retr_layernorm_fwd launches vs retr_linear_fwd_splitk_ln (split-K slabs +
slab_epilogue_ln, RETR_TUNE_ROWLN = 1) at 2 / 4 slices and the row-complete tile (ROWLN 2).
20 calls in a hipGraph, best of 5 replays.

    python tools/outproj_ln_micro.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from retr_amd import _lib  # noqa: E402
from retr_amd._lib import ptr  # noqa: E402

DEV = "cuda"


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn(s.cuda_stream)
    best = 1e30
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def main():
    lib = _lib.load()
    g = torch.Generator().manual_seed(0)
    for M, period in ((2048, 128), (6400, 400)):
        K = N = 256
        x = (torch.randn(M, K, generator=g) * 0.5).to(DEV).bfloat16()
        w = (torch.randn(N, K, generator=g) * 0.05).to(DEV).bfloat16()
        bias = torch.randn(N, generator=g).to(DEV)
        res = torch.randn(M, N, generator=g).to(DEV)
        gamma = (torch.rand(N, generator=g) + 0.5).to(DEV)
        beta = torch.randn(N, generator=g).to(DEV)
        pos = torch.randn(period, N, generator=g).to(DEV)
        y = torch.empty(M, N, device=DEV)
        ly = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ly2 = torch.empty_like(ly)
        mean = torch.empty(M, device=DEV)
        rstd = torch.empty(M, device=DEV)
        ws = torch.empty(4, M, N, device=DEV)

        def sep(st):
            rc = lib.retr_linear_fwd(1, ptr(x), K, ptr(w), K, ptr(bias), ptr(y), N, 1, M, N, K, 0,
                                     ptr(res), N, 0.1, 1234, st)
            assert rc == 0, lib.retr_last_error()
            rc = lib.retr_layernorm_fwd(1, ptr(y), N, ptr(gamma), ptr(beta), 1e-5, M, N, ptr(ly),
                                        N, ptr(ly2), ptr(pos), period, ptr(mean), ptr(rstd), st)
            assert rc == 0, lib.retr_last_error()

        res_t = {"separate": timed(sep)}
        for name, knob, splits in (("slab2", 1, 2), ("slab4", 1, 4), ("rowln", 2, 1)):
            d = _lib.LnOut(ptr(gamma), ptr(beta), 1e-5, 1, ptr(ly), ptr(ly2), N, ptr(pos), period,
                           ptr(mean), ptr(rstd))
            lib.retr_tune(32, knob)

            def fused(st, d=d, splits=splits):
                rc = lib.retr_linear_fwd_splitk_ln(1, ptr(x), K, ptr(w), K, ptr(bias), ptr(y), N,
                                                   M, N, K, 0, ptr(res), N, 0.1, 1234,
                                                   ptr(ws) if splits > 1 else None, splits,
                                                   ctypes.byref(d), st)
                assert rc == 0, lib.retr_last_error()
            res_t[name] = timed(fused)
            lib.retr_tune(32, 0)
        print(f"M{M} N256 K256 +LN: " + "  ".join(f"{k} {v:6.2f} us" for k, v in res_t.items()),
              flush=True)


if __name__ == "__main__":
    main()
