"""Phase timestamps inside dec_attn_row2_kernel (block 0, wave 0; wall_clock64 at 100 MHz) from
the -DRETR_DEC_TIMING build of the library in tools/_timing/ (build it with
`make -f tools/Makefile.timing`), cfg5 shapes (C 256, H 8, R 64).

    python tools/dec_phase.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_timing", "libretr_hip.so")
from retr_amd import ops  # noqa: E402
from retr_amd._lib import call, ptr  # noqa: E402

DEV = "cuda"
NAMES = ["start", "loads issued", "q in LDS", "softmax", "PV+shfl", "merged", "wo.dot",
         "LN done", "wq.dot", "sync", "stored"]


def main():
    lib = _lib.load()
    lib.retr_dec_timing_read.argtypes = [ctypes.c_void_p]
    C, H, T, S, R = 256, 8, 128, 196, 64
    g = torch.Generator().manual_seed(0)
    bf = torch.bfloat16

    def rnd(*s, dt=torch.float32, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(DEV).to(dt)

    q = rnd(R, C, dt=bf)
    kc, vc = rnd(R * T, C, dt=bf), rnd(R * T, C, dt=bf)
    kx, vx = rnd(64 * S, C, dt=bf), rnd(64 * S, C, dt=bf)
    kpm = torch.zeros(64, S, dtype=torch.uint8, device=DEV)
    x, xo = rnd(R, C), torch.empty(R, C, device=DEV)
    w, b = rnd(C, C, dt=bf, scale=0.06), rnd(C)
    gm, bt, pos = rnd(C) + 1, rnd(C), rnd(C)
    q2 = torch.empty(R, C, dtype=bf, device=DEV)
    st = ops._st()
    cases = {
        "self Lk64": lambda: call("retr_dec_attn_row", ptr(q), ptr(kc), ptr(vc), R, C, H, 64, T, 1,
                                  None, None, ptr(x), ptr(w), ptr(b), ptr(xo), ptr(gm), ptr(bt),
                                  1e-12, ptr(pos), ptr(w), ptr(b), ptr(q2), st),
        "cross S196": lambda: call("retr_dec_attn_row", ptr(q), ptr(kx), ptr(vx), R, C, H, S, S, 1,
                                   None, ptr(kpm), ptr(x), ptr(w), ptr(b), ptr(xo), ptr(gm),
                                   ptr(bt), 1e-12, None, None, None, ptr(q2), st),
    }
    out = (ctypes.c_longlong * 16)()
    for name, fn in cases.items():
        rows = []
        for rep in range(6):
            torch.cuda.synchronize()
            fn()
            torch.cuda.synchronize()
            lib.retr_dec_timing_read(ctypes.addressof(out))
            t = list(out)
            rows.append([(t[i] - t[0]) * 10 for i in range(11)])
        print(f"== {name} (ns since first instruction of wave 0, block 0; last 3 reps)")
        for i, n in enumerate(NAMES):
            # the cross-attention case has no next-layer q projection: its last three stamps are
            # never written (stale values from the previous case read negative)
            print(f"  {n:14s} " + " ".join(f"{r[i]:7d}" if r[i] >= 0 else "    n/a"
                                           for r in rows[-3:]))


if __name__ == "__main__":
    main()
