"""Phase timing of the fused bottleneck kernel from per-wave s_memrealtime stamps (100 MHz),
the BN_DIAG=9 build (tools/_ab/bn_diag9.so from tools/bn_micro.sh): for the first 4096 blocks,
mean per-wave time in phase A loop / A epilogue+barrier / B MFMAs / B epilogue+barrier /
C MFMAs / C epilogue, and the mean block lifetime.

    python tools/bn_phase.py tools/_ab/bn_diag9.so
"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from bn_micro import SHAPES, fn, run  # noqa: E402

DEV = "cuda"


def main():
    path = sys.argv[1]
    f = fn(path)
    lib = ctypes.CDLL(path)
    lib.retr_bn_prof.argtypes = [ctypes.c_void_p]
    st = torch.cuda.current_stream().cuda_stream
    names = ["A loop", "A epi+bar", "B mfma", "B epi+bar", "C mfma", "C epi"]
    for N, H, W, C, ds in SHAPES:
        x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
        w1 = (torch.randn(64, C, device=DEV) / C ** 0.5).to(torch.bfloat16)
        b1 = torch.randn(64, device=DEV) * 0.1
        w2 = (torch.randn(64, 3, 3, 64, device=DEV) / 24).to(torch.bfloat16)
        b2 = torch.randn(64, device=DEV) * 0.1
        K3 = 64 + (C if ds else 0)
        w3 = (torch.randn(256, K3, device=DEV) / K3 ** 0.5).to(torch.bfloat16)
        b3 = torch.randn(256, device=DEV) * 0.1
        y = torch.empty(N, H, W, 256, device=DEV, dtype=torch.bfloat16)
        for _ in range(3):
            run(f, x, w1, b1, w2, b2, w3, b3, ds, y, st)
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 8 * 8, dtype=np.uint64)
        assert lib.retr_bn_prof(buf.ctypes.data) == 0
        t = buf.reshape(4096, 8, 8)[:, :, :7].astype(np.int64)
        nb = min(4096, N * (H // 8) * (W // 16))
        t = t[:nb]
        d = np.diff(t, axis=2) * 10 / 1000.0          # us
        life = (t[:, :, 6].max(1) - t[:, :, 0].min(1)) * 10 / 1000.0
        span = (t[:, :, 6].max() - t[:, :, 0].min()) * 10 / 1000.0
        print(f"N{N} {H}x{W}x{C} ds{ds}: {nb} blocks, span {span:.1f} us, block life "
              f"{life.mean():.2f} us (p90 {np.percentile(life, 90):.2f})")
        for k, nm in enumerate(names):
            v = d[:, :, k]
            print(f"   {nm:12s} mean {v.mean():6.2f} us  p10 {np.percentile(v, 10):6.2f}  "
                  f"p90 {np.percentile(v, 90):6.2f}")


if __name__ == "__main__":
    main()
