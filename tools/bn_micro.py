"""Device time of retr_bottleneck_s1_fwd variants (stand-alone libraries built by
tools/bn_micro.sh) on the cfg2 layer1 shapes: N16 160x160, identity block (Cin 256) and the
first block (Cin 64, downsample folded in).  Every variant must produce the same bytes as the
first library listed; 20 launches captured in a hipGraph, best of 5 replays; achieved HBM GB/s
from the algorithmic bytes (x read once, y written once, weights once).

    python tools/bn_micro.py tools/_ab/bn_head.so tools/_ab/bn_cur.so ...
"""
import ctypes
import sys

import torch

DEV = "cuda"
SHAPES = [(16, 160, 160, 256, 0), (16, 160, 160, 64, 1)]


def fn(path):
    lib = ctypes.CDLL(path)
    f = lib.retr_bottleneck_s1_fwd
    P, I = ctypes.c_void_p, ctypes.c_int
    f.argtypes = [I, P, I, I, I, I, P, P, P, P, P, P, I, P, P]
    f.restype = I
    return f


def run(f, x, w1, b1, w2, b2, w3, b3, ds, y, st):
    N, H, W, C = x.shape
    rc = f(1, x.data_ptr(), N, H, W, C, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
           b2.data_ptr(), w3.data_ptr(), b3.data_ptr(), ds, y.data_ptr(), st)
    assert rc == 0, rc


def main():
    libs = sys.argv[1:]
    fns = [fn(p) for p in libs]
    torch.manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    for N, H, W, C, ds in SHAPES:
        x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
        w1 = (torch.randn(64, C, device=DEV) / C ** 0.5).to(torch.bfloat16)
        b1 = torch.randn(64, device=DEV) * 0.1
        w2 = (torch.randn(64, 3, 3, 64, device=DEV) / 24).to(torch.bfloat16)
        b2 = torch.randn(64, device=DEV) * 0.1
        K3 = 64 + (C if ds else 0)
        w3 = (torch.randn(256, K3, device=DEV) / K3 ** 0.5).to(torch.bfloat16)
        b3 = torch.randn(256, device=DEV) * 0.1
        byts = 2 * N * H * W * (C + 256) + 2 * (64 * C + 9 * 64 * 64 + 256 * K3)
        ref = None
        for path, f in zip(libs, fns):
            y = torch.empty(N, H, W, 256, device=DEV, dtype=torch.bfloat16)
            run(f, x, w1, b1, w2, b2, w3, b3, ds, y, st)
            torch.cuda.synchronize()
            same = "ref" if ref is None else ("bitwise" if torch.equal(y, ref) else
                                              f"DIFF max {(y.float() - ref.float()).abs().max():.3g}")
            ref = y if ref is None else ref
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                run(f, x, w1, b1, w2, b2, w3, b3, ds, y, s.cuda_stream)
                with torch.cuda.graph(g, stream=s):
                    for _ in range(20):
                        run(f, x, w1, b1, w2, b2, w3, b3, ds, y, s.cuda_stream)
            best = 1e9
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20)
            print(f"N{N} {H}x{W}x{C} ds{ds}  {path.split('/')[-1]:18s} {best * 1e3:8.1f} us "
                  f"{byts / best / 1e6:7.0f} GB/s  {same}", flush=True)


if __name__ == "__main__":
    main()
