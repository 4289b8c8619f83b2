"""Device time of the bf16 3x3 stride-1 convolutions of cfg2 (forward + ReLU, data gradient +
ReLU gate): the direct kernel's tile variants (RETR_TUNE_C3_TILE) vs the implicit GEMM
(RETR_TUNE_CONV3X3 = 1).  20 calls captured in a hipGraph, best of 5 replays; with --rounds R
the variants are timed R times interleaved and the minimum / median over rounds is printed
(variants 9-11 are 7 / 1 / 2 with the 144-byte halo rows of rounds 3-5).

    python tools/c3_micro.py [--variants 0,1,2,...] [--rounds 3]
"""
import statistics
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402

DEV = "cuda"
SHAPES = [(16, 80, 80, 128, 128), (16, 40, 40, 256, 256), (16, 20, 20, 512, 512)]


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    best = 1e30
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


def main():
    variants = [int(v) for v in (sys.argv[sys.argv.index("--variants") + 1].split(",")
                                 if "--variants" in sys.argv else "0,1,2,3,4,5,6,7,8".split(","))]
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 1
    lib = load()
    bf = torch.bfloat16
    for nb, H, W, C, Co in SHAPES:
        x = torch.randn(nb, H, W, C, device=DEV).to(bf)
        wf = (torch.randn(Co, 3, 3, C, device=DEV) * 0.05).to(bf)
        wt = (torch.randn(C, 3, 3, Co, device=DEV) * 0.05).to(bf)
        b = torch.randn(Co, device=DEV)
        y = torch.empty(nb, H, W, Co, device=DEV, dtype=bf)
        dy = torch.randn(nb, H, W, Co, device=DEV).to(bf)
        gate = torch.randn(nb, H, W, C, device=DEV).to(bf)
        dx = torch.empty(nb, H, W, C, device=DEV, dtype=bf)
        fl = 2.0 * nb * H * W * C * Co * 9
        for kind in ("fwd", "dgrad"):
            times = {v: [] for v in [-1] + variants}
            for _ in range(rounds):
                for v in [-1] + variants:
                    lib.retr_tune(21, 1 if v < 0 else 2)
                    lib.retr_tune(22, max(v, 0))
                    if kind == "fwd":
                        fn = lambda: call("retr_conv2d_fwd", 1, ptr(x), nb, H, W, C, ptr(wf), ptr(b),  # noqa: E731
                                          None, ptr(y), Co, 3, 3, 1, 1, 1, 1, stream())
                    else:
                        fn = lambda: call("retr_conv2d_dgrad", 1, ptr(dy), nb, H, W, C, ptr(wt),  # noqa: E731
                                          ptr(dx), Co, 3, 3, 1, 1, 1, None, ptr(gate), stream())
                    try:
                        times[v].append(timed(fn))
                    except Exception:   # noqa: BLE001
                        times[v].append(float("nan"))
            res = []
            for v, ts in times.items():
                us = min(ts)
                med = f"/med {statistics.median(ts):.1f}" if rounds > 1 else ""
                res.append(f"{'gemm' if v < 0 else 'v%d' % v}={us:.1f}{med}us/{fl / us / 1e6:.0f}TF")
            print(f"{kind:5s} N{nb} {H}x{W} {C}->{Co}: " + "  ".join(res), flush=True)
    lib.retr_tune(21, 0)
    lib.retr_tune(22, 0)


if __name__ == "__main__":
    main()
