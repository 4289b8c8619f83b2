"""A/B of the resident bf16 attention backward on the cfg2 shapes (encoder 400x400, cross
128x400, decoder causal 128x128; B 16, H 8, hd 32, dropout 0.1 with saved keep bits):
RETR_TUNE_ATTN_SPLIT 1 (one wave per 32 rows) vs 0 (even / odd key or query tiles on two
waves).  20 calls in a hipGraph, best of 5 replays.

    python tools/attn_bwd_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import load  # noqa: E402
from tools.attn_micro import SHAPES, timeit  # noqa: E402

DEV = "cuda"


def main():
    B, H, hd = 16, 8, 32
    bf = torch.bfloat16
    for Lq, Lk, causal in SHAPES:
        g = torch.Generator().manual_seed(0)
        C = H * hd
        q, k, v, do = (torch.randn(B * L, C, generator=g).to(DEV).to(bf) for L in (Lq, Lk, Lk, Lq))
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[: B // 2, Lk - Lk // 8:] = 1
        kpm = kpm.to(DEV)
        o = torch.empty(B * Lq, C, dtype=bf, device=DEV)
        lse = torch.empty(B * H * Lq, device=DEV)
        dq, dk, dv = (torch.empty_like(t) for t in (q, k, v))
        dm = ops.attn_dmask(B, H, Lq, Lk, 0.1, bf, hd, DEV)
        ops.k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, causal, 0.1, 7, lse, None, dm)
        line = f"{Lq}x{Lk} c{causal}:"
        flop = 10.0 * B * H * Lq * Lk * hd * (0.5 if causal else 1.0)
        for split in (1, 0):
            load().retr_tune(10, split)
            t = timeit(lambda: ops.k_attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk,
                                                   hd, kpm, causal, 0.1, 7, dm))
            line += f"  split{'off' if split == 1 else 'on '} {t:6.1f} us {flop / t / 1e6:6.1f} TF/s"
        load().retr_tune(10, 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
