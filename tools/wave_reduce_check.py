"""Bitwise check of common.hpp's crossbar-free wave_sum / wave_max against the __shfl_xor
butterfly (tools/wave_reduce_check.hip, built into tools/_ab/wave_reduce_check.so):
random normal data at several scales, with signed zeros and infinities mixed in.

    python tools/wave_reduce_check.py
"""
import ctypes
import os
import sys

import torch

path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "_ab",
                                                          "wave_reduce_check.so")
lib = ctypes.CDLL(path)
lib.wave_reduce_check.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
g = torch.Generator(device="cuda").manual_seed(0)
total = [0, 0, 0, 0]
for scale in (1e-30, 1e-3, 1.0, 1e3, 1e30):
    n = 1 << 22
    x = torch.randn(n, device="cuda", generator=g) * scale
    r = torch.rand(n, device="cuda", generator=g)
    x[r < 0.05] = 0.0
    x[(r >= 0.05) & (r < 0.1)] = -0.0
    x[(r >= 0.1) & (r < 0.101)] = float("inf")
    x[(r >= 0.101) & (r < 0.102)] = -float("inf")
    bad = torch.zeros(4, dtype=torch.int32, device="cuda")
    assert lib.wave_reduce_check(x.data_ptr(), n, bad.data_ptr()) == 0
    b = bad.tolist()
    total = [t + x for t, x in zip(total, b)]
    print(f"scale {scale:g}: sum mismatches {b[0]}, max {b[1]}, xor partners {b[2]}, ascending "
          f"butterfly {b[3]} of {n} lanes", flush=True)
print("OK" if not any(total) else "MISMATCH")
sys.exit(0 if not any(total) else 1)
