"""Device-time micro-benchmark of the bf16 attention kernels on the cfg2 shapes (encoder
self-attention 400x400, decoder cross 128x400, decoder causal 128x128; B 16, H 8, hd 32,
dropout 0.1, a padded key mask), streaming (mode 1) vs LDS-resident (mode 2) kernels.
20 calls captured into a hipGraph, best of 5 replays.

    python tools/attn_micro.py                    # the table
    python tools/attn_micro.py fwd 400 400 0 2    # one variant (for rocprofv3 --pmc runs)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import ops  # noqa: E402
from retr_amd._lib import load  # noqa: E402

DEV = "cuda"
SHAPES = [(400, 400, 0), (128, 400, 0), (128, 128, 1)]


def timeit(fn, n=20):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(n):
            fn()
    best = float("inf")
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def setup(Lq, Lk, causal, B=16, H=8, hd=32):
    g = torch.Generator().manual_seed(0)
    C = H * hd
    bf = torch.bfloat16
    q, k, v, do = (torch.randn(B * L, C, generator=g).to(DEV).to(bf) for L in (Lq, Lk, Lk, Lq))
    kpm = torch.zeros(B, Lk, dtype=torch.uint8)
    kpm[: B // 2, Lk - Lk // 8:] = 1
    kpm = kpm.to(DEV)
    o = torch.empty(B * Lq, C, dtype=bf, device=DEV)
    lse = torch.empty(B * H * Lq, device=DEV)
    dq, dk, dv = (torch.empty_like(t) for t in (q, k, v))
    fwd = lambda: ops.k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, causal, 0.1, 7, lse)  # noqa: E731
    bwd = lambda: ops.k_attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, hd, kpm,  # noqa: E731
                                      causal, 0.1, 7)
    fwd()
    return fwd, bwd, 4.0 * B * H * Lq * Lk * hd * (0.5 if causal else 1.0)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "bsplit":   # backward split (RETR_TUNE_ATTN_SPLIT)
        for Lq, Lk, causal in SHAPES:
            fwd, bwd, fl = setup(Lq, Lk, causal)
            out = []
            for sk in (0, 1, 3, 4):
                load().retr_tune(10, sk)
                t = timeit(bwd)
                out.append(f"split{sk}: {t:6.2f} us {2.5 * fl / t / 1e6:5.1f} TF/s")
            load().retr_tune(10, 0)
            print(f"bwd Lq{Lq:4d} Lk{Lk:4d} causal{causal} | " + " | ".join(out), flush=True)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "fsplit":   # forward key split (RETR_TUNE_ATTN_FSPLIT)
        for Lq, Lk, causal in SHAPES:
            fwd, bwd, fl = setup(Lq, Lk, causal)
            out = []
            for fs in (0, 1, 2, 3, 4):
                load().retr_tune(12, fs)
                t = timeit(fwd)
                out.append(f"fs{fs}: {t:6.2f} us {fl / t / 1e6:5.1f} TF/s")
            load().retr_tune(12, 0)
            print(f"fwd Lq{Lq:4d} Lk{Lk:4d} causal{causal} | " + " | ".join(out), flush=True)
        return
    if len(sys.argv) > 1:
        which, Lq, Lk, causal, mode = sys.argv[1], *map(int, sys.argv[2:6])
        load().retr_tune(5, mode)
        fwd, bwd, fl = setup(Lq, Lk, causal)
        t = timeit(fwd if which == "fwd" else bwd)
        print(f"{which} {Lq}x{Lk} c{causal} mode {mode}: {t:.2f} us")
        return
    for Lq, Lk, causal in SHAPES:
        for mode in (1, 2):
            load().retr_tune(5, mode)
            fwd, bwd, fl = setup(Lq, Lk, causal)
            tf, tb = timeit(fwd), timeit(bwd)
            print(f"Lq{Lq:4d} Lk{Lk:4d} causal{causal} mode{mode}: fwd {tf:7.2f} us "
                  f"{fl / tf / 1e6:6.1f} TF/s   bwd {tb:7.2f} us {2.5 * fl / tb / 1e6:6.1f} TF/s",
                  flush=True)
    load().retr_tune(5, 0)


if __name__ == "__main__":
    main()
