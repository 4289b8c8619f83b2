"""Device time of retr_stem_pool_fwd variants (stand-alone libraries built by tools/stem_micro.sh)
at the cfg2 stem shape (N16, s2d input 320x320x16 -> pooled 160x160x64) and the cfg5 decode
shape (N64, 112x112).  Every variant must produce the same bytes as the first library listed;
20 launches captured in a hipGraph, best of 5 replays; achieved GB/s from the algorithmic bytes
(s2d input once, pooled output once).  A library exporting retr_stem_prof (STEM_DIAG=9) also
prints the mean per-wave phase times of the first 4096 blocks.

    python tools/stem_micro.py tools/_ab/stem_cur.so tools/_ab/stem_diag9.so ...
"""
import ctypes
import sys

import numpy as np
import torch

DEV = "cuda"
SHAPES = [(16, 320, 320), (64, 112, 112)]
PHASES = ["patch+w0", "mfma0", "pool0", "w1+bar", "mfma1", "pool1"]


def fn(path):
    lib = ctypes.CDLL(path)
    f = lib.retr_stem_pool_fwd
    P, I = ctypes.c_void_p, ctypes.c_int
    f.argtypes = [I, P, I, I, I, P, P, P, I, P]
    f.restype = I
    return lib, f


def main():
    libs = sys.argv[1:]
    fns = [fn(p) for p in libs]
    torch.manual_seed(0)
    for N, H2, W2 in SHAPES:
        x = torch.randn(N, H2, W2, 16, device=DEV)
        x[..., 12:] = 0
        x = x.to(torch.bfloat16)
        w = (torch.randn(64, 256, device=DEV) / 16).to(torch.bfloat16)
        b = torch.randn(64, device=DEV) * 0.1
        PH, PW = (H2 - 1) // 2 + 1, (W2 - 1) // 2 + 1
        byts = 2 * (N * H2 * W2 * 16 + N * PH * PW * 64 + 64 * 256)
        ref = None
        for path, (lib, f) in zip(libs, fns):
            y = torch.empty(N, PH, PW, 64, device=DEV, dtype=torch.bfloat16)

            def run(st):
                assert f(1, x.data_ptr(), N, H2, W2, w.data_ptr(), b.data_ptr(), y.data_ptr(),
                         64, st) == 0

            run(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            same = "ref" if ref is None else ("bitwise" if torch.equal(y, ref) else
                                              f"DIFF max {(y.float() - ref.float()).abs().max():.3g}")
            ref = y if ref is None else ref
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                run(s.cuda_stream)
                with torch.cuda.graph(g, stream=s):
                    for _ in range(20):
                        run(s.cuda_stream)
            best = 1e9
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20)
            print(f"N{N} {H2}x{W2}  {path.split('/')[-1]:18s} {best * 1e3:8.1f} us "
                  f"{byts / best / 1e6:7.0f} GB/s  {same}", flush=True)
            if hasattr(lib, "retr_stem_prof"):
                lib.retr_stem_prof.argtypes = [ctypes.c_void_p]
                buf = np.zeros(4096 * 8 * 8, dtype=np.uint64)
                run(torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                lib.retr_stem_prof(buf.ctypes.data)
                t = buf.reshape(4096, 8, 8).astype(np.float64)[..., :7] * 10.0   # ns (100 MHz)
                nblk = min(4096, (N * ((PH + 7) // 8) * ((PW + 15) // 16)))
                t = t[:nblk]
                d = np.diff(t, axis=2).mean(axis=(0, 1)) / 1e3
                life = (t[..., 6].max(axis=1) - t[..., 0].min(axis=1)).mean() / 1e3
                print("   phases (us/wave): " + "  ".join(f"{n} {v:.2f}" for n, v in zip(PHASES, d))
                      + f"  | block life {life:.2f} us", flush=True)


if __name__ == "__main__":
    main()
