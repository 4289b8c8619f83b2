"""Per-block timestamps of the resident attention backward kernels (dq3 = 0, dkdv3 = 1) from the
-DRETR_ATTN_TIMING build (make -f tools/Makefile.timing_attn): for the cfg2 shapes, the kernel
span, the block start spread (rounds of blocks), and per-block prologue (LDS-DMA issue +
drain) and tile-loop durations (wall_clock64, 100 MHz).

    python tools/attn_phase.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_timing_attn",
                             "libretr_hip.so")
from retr_amd import ops  # noqa: E402

DEV = "cuda"


def main():
    lib = _lib.load()
    lib.retr_attn_timing_read.argtypes = [ctypes.c_void_p]
    B, H, hd = 16, 8, 32
    bf = torch.bfloat16
    for Lq, Lk, causal in ((400, 400, 0), (128, 400, 0)):
        C = H * hd
        g = torch.Generator().manual_seed(0)
        q, o, do = (torch.randn(B * Lq, C, generator=g).to(DEV).to(bf) for _ in range(3))
        k, v = (torch.randn(B * Lk, C, generator=g).to(DEV).to(bf) for _ in range(2))
        lse = torch.randn(B * H * Lq, generator=g).to(DEV).abs() + 5
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        kpm = torch.zeros(B, Lk, dtype=torch.uint8, device=DEV)
        for _ in range(3):
            ops.k_attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, hd, kpm, causal,
                                0.1, 1234)
        torch.cuda.synchronize()
        buf = np.zeros(2 * 8192 * 3, dtype=np.int64)
        lib.retr_attn_timing_read(buf.ctypes.data)
        t = buf.reshape(2, 8192, 3)
        for kname, kk in (("dq3", 0), ("dkdv3", 1)):
            x = t[kk]
            x = x[x[:, 0] > 0]
            if len(x) == 0:
                print(f"Lq{Lq} Lk{Lk} {kname}: no stamps (streaming kernel ran)")
                continue
            t0 = x[:, 0].min()
            st = (x[:, 0] - t0) * 10 / 1e3          # us
            pro = (x[:, 1] - x[:, 0]) * 10 / 1e3
            loop = (x[:, 2] - x[:, 1]) * 10 / 1e3
            span = (x[:, 2].max() - t0) * 10 / 1e3
            q = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 50, 90, 100))  # noqa
            print(f"Lq{Lq} Lk{Lk} {kname}: {len(x)} blocks, span(first start->last loop end) "
                  f"{span:.2f} us | start p0/50/90/100 {q(st)} | prologue {q(pro)} | "
                  f"tile loop {q(loop)}", flush=True)


if __name__ == "__main__":
    main()
