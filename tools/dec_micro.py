"""Micro-timings of the fused decode kernels (csrc/decode.hip) in isolation: HIP events around
100 back-to-back launches, cfg5 shapes (C 256, H 8, S 196, F 2048), R rows."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import call, ptr  # noqa: E402

DEV = "cuda"


def timeit(fn, n=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    C, H, T, S, F = 256, 8, 128, 196, 2048
    g = torch.Generator().manual_seed(0)
    bf = torch.bfloat16

    def rnd(*s, dt=torch.float32, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(DEV).to(dt)

    for R in (64, 320):
        q = rnd(R, C, dt=bf)
        kc, vc = rnd(R * T, C, dt=bf), rnd(R * T, C, dt=bf)
        kx, vx = rnd(64 * S, C, dt=bf), rnd(64 * S, C, dt=bf)
        kpm = torch.zeros(64, S, dtype=torch.uint8, device=DEV)
        x, xo = rnd(R, C), torch.empty(R, C, device=DEV)
        w, b = rnd(C, C, dt=bf, scale=0.06), rnd(C)
        gm, bt, pos = rnd(C) + 1, rnd(C), rnd(C)
        q2 = torch.empty(R, C, dtype=bf, device=DEV)
        K = R // 64
        st = ops._st()
        res = {}
        for Lk in (1, 64, 127):
            res[f"self Lk{Lk}"] = timeit(lambda: call(
                "retr_dec_attn_row", ptr(q), ptr(kc), ptr(vc), R, C, H, Lk, T, 1, None, None,
                ptr(x), ptr(w), ptr(b), ptr(xo), ptr(gm), ptr(bt), 1e-12, ptr(pos), ptr(w),
                ptr(b), ptr(q2), st))
        res["self Lk127 no-wq"] = timeit(lambda: call(
            "retr_dec_attn_row", ptr(q), ptr(kc), ptr(vc), R, C, H, 127, T, 1, None, None,
            ptr(x), ptr(w), ptr(b), ptr(xo), ptr(gm), ptr(bt), 1e-12, None, None, None, ptr(q2),
            st))
        res["cross S196"] = timeit(lambda: call(
            "retr_dec_attn_row", ptr(q), ptr(kx), ptr(vx), R, C, H, S, S, K, None, ptr(kpm),
            ptr(x), ptr(w), ptr(b), ptr(xo), ptr(gm), ptr(bt), 1e-12, None, None, None, ptr(q2),
            st))
        w3 = rnd(3 * C, C, dt=bf, scale=0.06)
        b3 = rnd(3 * C)
        res["dec_gemm qkv"] = timeit(lambda: call(
            "retr_dec_gemm", ptr(q), ptr(q), R, C, ptr(w3), ptr(b3), 3 * C, ptr(q2), C, 1,
            ptr(kc), T * C, 1, ptr(vc), T * C, 0, C, 0, st))
        w1, w2 = rnd(F, C, dt=bf, scale=0.06), rnd(C, F, dt=bf, scale=0.02)
        b1 = rnd(F)
        slabs = torch.empty(F // 32, R, C, device=DEV)
        res["dec_ffn"] = timeit(lambda: call(
            "retr_dec_ffn", ptr(q), R, C, ptr(w1), ptr(b1), ptr(w2), F, ptr(slabs), st))
        res["dec_rows 64 slabs"] = timeit(lambda: call(
            "retr_dec_rows", ptr(x), ptr(slabs), F // 32, ptr(b), R, C, ptr(xo), ptr(gm),
            ptr(bt), 1e-12, ptr(pos), ptr(q2), ptr(q2), st))
        res["dec_rows no slabs"] = timeit(lambda: call(
            "retr_dec_rows", ptr(x), None, 0, None, R, C, None, ptr(gm), ptr(bt), 1e-12,
            ptr(pos), ptr(q2), ptr(q2), st))
        res["empty-ish ln"] = timeit(lambda: call(
            "retr_layernorm_fwd", 1, ptr(x), C, ptr(gm), ptr(bt), 1e-12, R, C, ptr(q2), C, None,
            None, 1, None, None, st))
        for k, v in res.items():
            print(f"R={R:4d} {k:22s} {v:8.2f} us/launch", flush=True)


if __name__ == "__main__":
    main()
