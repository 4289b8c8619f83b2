"""Device-time sweep of the large-GEMM tile choice (retr_tune RETR_TUNE_BIG_TILE) on the
memory-heavy ResNet-50 convolutions of cfg2 (batch 16, 640x640 input): 1x1 convolutions over
the 160x160 / 80x80 / 40x40 maps with residual or addend, the stem and strided data gradients.
20 calls captured in a hipGraph, best of 5 replays; achieved HBM GB/s from the operand and
output bytes (algorithmic traffic).

    python tools/conv_micro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402

DEV = "cuda"
BF = 1
# (kind, N, H, W, C, Co, k, s, p, with residual/addend)
SHAPES = [("fwd", 16, 160, 160, 64, 256, 1, 1, 0, 1), ("fwd", 16, 160, 160, 64, 256, 1, 1, 0, 0),
          ("fwd", 16, 80, 80, 128, 512, 1, 1, 0, 1), ("fwd", 16, 40, 40, 256, 1024, 1, 1, 0, 1),
          ("fwd", 16, 160, 160, 256, 64, 1, 1, 0, 0), ("fwd", 16, 160, 160, 64, 64, 3, 1, 1, 0),
          ("fwd", 16, 640, 640, 8, 64, 7, 2, 3, 0),
          ("fwd", 16, 20, 20, 512, 512, 3, 1, 1, 0), ("fwd", 16, 20, 20, 2048, 512, 1, 1, 0, 0),
          ("fwd", 16, 20, 20, 512, 2048, 1, 1, 0, 1), ("fwd", 16, 40, 40, 512, 512, 3, 2, 1, 0),
          ("dgrad", 16, 20, 20, 512, 512, 3, 1, 1, 0), ("dgrad", 16, 20, 20, 512, 2048, 1, 1, 0, 1),
          ("dgrad", 16, 20, 20, 2048, 512, 1, 1, 0, 1),
          ("dgrad", 16, 40, 40, 1024, 256, 1, 1, 0, 1), ("dgrad", 16, 80, 80, 512, 128, 1, 1, 0, 1),
          ("dgrad", 16, 80, 80, 512, 1024, 1, 2, 0, 1), ("dgrad", 16, 40, 40, 1024, 2048, 1, 2, 0, 1),
          ("wgrad", 16, 40, 40, 256, 256, 3, 1, 1, 0), ("wgrad", 16, 80, 80, 128, 128, 3, 1, 1, 0),
          ("wgrad", 16, 20, 20, 512, 512, 3, 1, 1, 0), ("wgrad", 16, 40, 40, 256, 1024, 1, 1, 0, 0),
          ("wgrad", 16, 40, 40, 512, 512, 3, 2, 1, 0), ("wgrad", 16, 80, 80, 256, 256, 3, 2, 1, 0),
          ("wgrad", 16, 80, 80, 128, 512, 1, 1, 0, 0)]


VARIANTS = [(0, 0), (1, 0), (2, 0), (4, 0), (5, 0), (6, 0)]
WGRAD_PLANS = [0, 1, 7, 10, 12, 14, 16]


def r50_shapes(N=16, res=640):
    """Every distinct forward / data-gradient convolution of the cfg2 ResNet-50 step (layer1
    frozen: forward only), with residual / addend where the model fuses one."""
    out = set()
    H = res // 4
    cin = 64
    for li, (planes, blocks, stride) in enumerate(((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))):
        train = li > 0
        for b in range(blocks):
            s = stride if b == 0 else 1
            Ho = H // s
            convs = [(cin, planes, 1, 1, 0, H, 0), (planes, planes, 3, s, 1, H, 0),
                     (planes, planes * 4, 1, 1, 0, Ho, 1)]
            if b == 0:
                convs.append((cin, planes * 4, 1, s, 0, H, 0))
            for C, Co, k, st, pd, Hin, res_ in convs:
                out.add(("fwd", N, Hin, Hin, C, Co, k, st, pd, res_))
                if train:
                    out.add(("dgrad", N, Hin, Hin, C, Co, k, st, pd, 1))
            cin = planes * 4
            H = Ho
    return sorted(out, key=lambda t: (t[0], -t[2], t[4], t[5]))


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


def stem(N=16, H=640):
    """Legacy stem (NHWC8 + 7x7 stride-2) vs the space-to-depth stem (s2d16 + 4x4 stride-1),
    conversion + conv per variant of the big-GEMM tile."""
    bf = torch.bfloat16
    img = torch.randn(N, 3, H, H, device=DEV)
    w = (torch.randn(64 * 7 * 7 * 8, device=DEV) * 0.05).to(bf)
    w2 = (torch.randn(64 * 4 * 4 * 16, device=DEV) * 0.05).to(bf)
    b = torch.randn(64, device=DEV)
    x8 = torch.empty(N * H * H * 8, dtype=bf, device=DEV)
    xs = torch.empty(N * H * H * 4, dtype=bf, device=DEV)
    OH = H // 2
    y = torch.empty(N * OH * OH * 64, dtype=bf, device=DEV)
    fl = 2.0 * N * OH * OH * 64 * 147
    cases = {
        "nhwc8": lambda: call("retr_nchw_to_nhwc", BF, ptr(img), ptr(x8), N, 3, H, H, 8, stream()),
        "s2d16": lambda: call("retr_nchw_to_s2d16", ptr(img), ptr(xs), N, 3, H, H, stream()),
    }
    for name, fn in cases.items():
        print(f"stem  {name:6s} conversion {timeit(fn):7.1f}us", flush=True)
    for tile in (0, 1, 2, 4, 6):
        load().retr_tune(6, tile)
        t7 = timeit(lambda: call("retr_conv2d_fwd", BF, ptr(x8), N, H, H, 8, ptr(w), ptr(b), None,
                                 ptr(y), 64, 7, 7, 2, 3, 1, 1, stream()))
        t4 = timeit(lambda: call("retr_conv2d_fwd_out", BF, ptr(xs), N, OH, OH, 16, ptr(w2),
                                 ptr(b), None, ptr(y), 64, 4, 4, 1, 2, 1, OH, OH, 1, stream()))
        print(f"stem  t{tile}: 7x7s2 {t7:7.1f}us {fl / t7 / 1e6:4.0f}TF | s2d 4x4 {t4:7.1f}us "
              f"{fl / t4 / 1e6:4.0f}TF", flush=True)
    load().retr_tune(6, 0)


def main():
    only = sys.argv[1] if len(sys.argv) > 1 else None
    small = len(sys.argv) > 2  # only the 20x20 / 40x40 (layer4) shapes
    bf = torch.bfloat16
    global VARIANTS
    if only == "stem":
        stem()
        return
    shapes = SHAPES
    if os.environ.get("RETR_VARIANTS"):   # e.g. RETR_VARIANTS=0,6,8,13 (RETR_TUNE_BIG_TILE values)
        VARIANTS = [(int(t), 0) for t in os.environ["RETR_VARIANTS"].split(",")]
    if only == "r50":
        shapes = r50_shapes()
        if not os.environ.get("RETR_VARIANTS"):
            VARIANTS = ([(0, 0), (13, 0), (14, 0)] if os.environ.get("RETR_SWEEP_S1")
                        else [(0, 0), (4, 0), (6, 0)])
    if only == "wtile":   # every cfg2 weight-gradient conv, 128x128 vs 64x64 tile
        shapes = sorted({("wgrad",) + t[1:9] + (0,) for t in r50_shapes() if t[0] == "dgrad"},
                        key=lambda t: (-t[2], t[4], t[5]))
    for kind, N, H, W, C, Co, k, s, p, extra in shapes:
        if only and only not in ("all", "r50", "wtile") and kind != only:
            continue
        if small and H > 40:
            continue
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N * H * W * C, device=DEV).to(bf)
        w = (torch.randn(Co * k * k * C, device=DEV) * 0.05).to(bf)
        b = torch.randn(Co, device=DEV)
        y = torch.empty(N * OH * OW * Co, dtype=bf, device=DEV)
        if kind == "fwd":
            res = torch.randn(N * OH * OW * Co, device=DEV).to(bf) if extra else None
            fn = lambda: call("retr_conv2d_fwd", BF, ptr(x), N, H, W, C, ptr(w), ptr(b),  # noqa: E731
                              ptr(res), ptr(y), Co, k, k, s, p, 1, 1, stream())
            nbytes = 2 * (x.numel() + y.numel() * (2 if extra else 1) + w.numel())
        elif kind == "wgrad":
            dy = torch.randn(N * OH * OW * Co, device=DEV).to(bf)
            grad = torch.empty(Co * C * k * k, device=DEV)

            def make_fn():
                sp = load().retr_conv2d_wgrad_splits(BF, N, H, W, C, Co, k, k, s, p, 1)
                ws = torch.empty(sp * Co * k * k * C, device=DEV)

                def fn():
                    call("retr_conv2d_wgrad", BF, ptr(dy), ptr(x), N, H, W, C, ptr(ws), Co, k, k,
                         s, p, 1, stream())
                    call("retr_conv_wgrad_unpack", ptr(ws), None, ptr(grad), Co, C, C, k, k, 0,
                         sp, stream())
                return fn, sp
            nbytes = 2 * (dy.numel() + x.numel())
        else:
            dy = torch.randn(N * OH * OW * Co, device=DEV).to(bf)
            add = torch.randn(N * H * W * C, device=DEV).to(bf) if extra else None
            dx = torch.empty(N * H * W * C, dtype=bf, device=DEV)
            fn = lambda: call("retr_conv2d_dgrad", BF, ptr(dy), N, H, W, C, ptr(w), ptr(dx), Co,  # noqa: E731
                              k, k, s, p, 1, ptr(add), None, stream())
            nbytes = 2 * (dy.numel() + dx.numel() * (2 if extra else 1) + w.numel())
        fl = 2.0 * N * OH * OW * Co * k * k * C
        out = []
        if kind == "wgrad":
            # split-K plan: 0 cost model (default), 1 legacy ceil(512 / tiles), >= 2 forced
            for tile in (2, 1):
                for plan in (WGRAD_PLANS if only != "wtile" else [0]):
                    load().retr_tune(8, plan)
                    load().retr_tune(9, tile)
                    fn, sp = make_fn()
                    t = timeit(fn)
                    out.append(f"{'t64' if tile == 1 else 't128'}/plan{plan}/s{sp}:{t:7.1f}us "
                               f"{fl / t / 1e6:4.0f}TF")
            load().retr_tune(8, 0)
            load().retr_tune(9, 0)
        for tile, nt in (VARIANTS if kind != "wgrad" else []):
            load().retr_tune(6, tile)
            load().retr_tune(7, nt)
            try:
                t = timeit(fn)
            except RuntimeError as e:   # a tile the shape cannot use
                out.append(f"t{tile}{'nt' if nt else ''}: -- ({str(e)[:30]})")
                continue
            out.append(f"t{tile}{'nt' if nt else ''}:{t:7.1f}us {nbytes / t / 1e3:5.0f}GB/s "
                       f"{fl / t / 1e6:4.0f}TF")
        load().retr_tune(6, 0)
        load().retr_tune(7, 0)
        print(f"{kind:5s} N{N} {H}x{W}x{C}->{Co} k{k}s{s} x{extra} | " + " | ".join(out),
              flush=True)


if __name__ == "__main__":
    main()
