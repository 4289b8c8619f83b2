"""Reference points for the GEMM core: hipBLASLt (torch.mm, bf16 -> bf16) vs retr_linear_fwd /
retr_linear_fwd_splitk on the cfg2 linear shapes and a dense 4k GEMM; 20 calls in a hipGraph,
best of 5 replays.  Measurement only (the product path never calls hipBLASLt).

    python tools/blas_ref.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd._lib import call, load, ptr, stream  # noqa: E402
from tools.conv_micro import timeit  # noqa: E402

SHAPES = [(4096, 4096, 4096), (6400, 256, 2048), (2048, 256, 2048), (6400, 2048, 256),
          (2048, 2048, 256), (6400, 256, 256), (2048, 256, 256), (6400, 768, 256),
          (2048, 30528, 512), (25600, 256, 2304), (102400, 512, 128)]


def main():
    bf = torch.bfloat16
    for M, N, K in SHAPES:
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        y = torch.empty(M, N, device="cuda", dtype=bf)
        wt = w.t()
        tb = timeit(lambda: torch.mm(x, wt, out=y))
        tr = timeit(lambda: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, None, ptr(y), N,
                                 0, M, N, K, 0, None, 0, 0.0, 0, stream()))
        s = load().retr_linear_splits(1, M, N, K)
        line = (f"M{M} N{N} K{K}: hipBLASLt {tb:7.1f} us {2 * M * N * K / tb / 1e6:5.0f} TF | "
                f"retr {tr:7.1f} us {2 * M * N * K / tr / 1e6:5.0f} TF")
        if s > 1:
            ws = torch.empty(s * M * N, device="cuda", dtype=torch.float32)
            ts = timeit(lambda: call("retr_linear_fwd_splitk", 1, ptr(x), K, ptr(w), K, None,
                                     ptr(y), N, 0, M, N, K, 0, None, 0, 0.0, 0, ptr(ws), s,
                                     stream()))
            line += f" | retr split{s} {ts:7.1f} us {2 * M * N * K / ts / 1e6:5.0f} TF"
        for v in [int(t) for t in os.environ.get("RETR_VARIANTS", "").split(",") if t]:
            load().retr_tune(6, v)           # RETR_TUNE_BIG_TILE: launch_big tile override
            tv = timeit(lambda: call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, None, ptr(y),
                                     N, 0, M, N, K, 0, None, 0, 0.0, 0, stream()))
            load().retr_tune(6, 0)
            line += f" | t{v} {tv:7.1f} us {2 * M * N * K / tv / 1e6:5.0f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
