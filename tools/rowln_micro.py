"""Device time of retr_linear_fwd_splitk_ln variants (RETR_TUNE_ROWLN) on the cfg2 FFN
down-projection shapes (M 6400 / 2048 tokens, K 2048 -> N 256, bias, dropout 0.1, fp32
residual, LayerNorm + position outputs): 1 = split-K slabs + slab_epilogue_ln (round 4-5),
2 / 3 / 4 = the row-complete 32 x 256 tile with the LayerNorm in its epilogue (2 / 3 / 4-stage
ring), 5 = its 64 x 256 8-wave variant.  20 calls in a hipGraph, best of 5 replays; every
variant's outputs against variant 1's (fp32 reassociation only).

    python tools/rowln_micro.py
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
KNOB = 32                      # RETR_TUNE_ROWLN


def main():
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(0)
    for M, period in ((6400, 400), (2048, 128)):
        K, N, splits = 2048, 256, 4
        x = (torch.randn(M, K, generator=g) * 0.5).to(DEV).bfloat16()
        w = (torch.randn(N, K, generator=g) * 0.02).to(DEV).bfloat16()
        bias = torch.randn(N, generator=g).to(DEV)
        res = torch.randn(M, N, generator=g).to(DEV)
        gamma = (torch.rand(N, generator=g) + 0.5).to(DEV)
        beta = torch.randn(N, generator=g).to(DEV)
        pos = torch.randn(period, N, generator=g).to(DEV)
        ws = torch.empty(splits, M, N, device=DEV)
        outs = {}
        for v in (1, 2, 3, 4, 5):
            y = torch.empty(M, N, device=DEV)
            ly = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            ly2 = torch.empty_like(ly)
            mean = torch.empty(M, device=DEV)
            rstd = torch.empty(M, device=DEV)
            d = _lib.LnOut(ptr(gamma), ptr(beta), 1e-5, 1, ptr(ly), ptr(ly2), N, ptr(pos), period,
                           ptr(mean), ptr(rstd))
            lib.retr_tune(KNOB, v)

            def call():
                rc = lib.retr_linear_fwd_splitk_ln(1, ptr(x), K, ptr(w), K, ptr(bias), ptr(y), N,
                                                   M, N, K, 0, ptr(res), N, 0.1, 1234, ptr(ws),
                                                   splits, ctypes.byref(d), st)
                assert rc == 0, lib.retr_last_error()

            call()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                st_s = s.cuda_stream

                def call_s():
                    rc = lib.retr_linear_fwd_splitk_ln(1, ptr(x), K, ptr(w), K, ptr(bias), ptr(y),
                                                       N, M, N, K, 0, ptr(res), N, 0.1, 1234,
                                                       ptr(ws), splits, ctypes.byref(d), st_s)
                    assert rc == 0
                with torch.cuda.graph(gr, stream=s):
                    for _ in range(20):
                        call_s()
            torch.cuda.current_stream().wait_stream(s)
            best = 1e9
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gr.replay()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
            outs[v] = (y.clone(), ly.float().clone(), ly2.float().clone(), mean.clone(),
                       rstd.clone())
            err = max(((a - b).abs().max() / b.abs().max()).item()
                      for a, b in zip(outs[v], outs[1]))
            flops = 2.0 * M * N * K
            print(f"M{M} N{N} K{K} +LN  variant {v}: {best:7.2f} us  {flops / best / 1e6:7.1f} TF/s"
                  f"  max rel diff vs 1: {err:.2e}", flush=True)
        lib.retr_tune(KNOB, 0)


if __name__ == "__main__":
    main()
