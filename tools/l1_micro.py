"""Layer-1 convs at cfg2 (N16 160x160, frozen, forward only): HIP-event time of each under every
large-GEMM tile knob (RETR_TUNE_BIG_TILE; 0 = built-in rule)."""
import math
import torch
from retr_amd import ops
from retr_amd._lib import call, ptr, load

DEV, bf = "cuda", torch.bfloat16


def timeit(fn, reps=40):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    N, H, W = 16, 160, 160
    st = ops._st()
    for (C, Co, k, res) in [(64, 256, 1, True), (256, 64, 1, False), (64, 64, 3, False),
                            (64, 64, 1, False)]:
        x = torch.randn(N, H, W, C, device=DEV).to(bf)
        w = (torch.randn(Co, k, k, C, device=DEV) / math.sqrt(C * k * k)).to(bf)
        b = torch.randn(Co, device=DEV)
        r = torch.randn(N, H, W, Co, device=DEV).to(bf) if res else None
        y = torch.empty(N, H, W, Co, dtype=bf, device=DEV)

        def f():
            call("retr_conv2d_fwd", ops.dcode(bf), ptr(x), N, H, W, C, ptr(w), ptr(b), ptr(r),
                 ptr(y), Co, k, k, 1, k // 2, 1, 1, st)

        byts = 2 * N * H * W * (C + Co * (2 if res else 1))
        line = f"N{N} {H}x{W}x{C}->{Co} k{k} res{int(res)}:"
        for knob in (0, 1, 2, 4, 6, 7, 8, 9):
            load().retr_tune(6, knob)
            t = timeit(f)
            line += f" | t{knob} {t:6.1f} us {byts / t / 1e3:5.0f} GB/s"
        load().retr_tune(6, 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
