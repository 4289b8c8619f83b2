"""Bottleneck tails at cfg2 (first block of each layer): fused retr_conv1x1_fwd_cat vs the
unfused downsample conv + conv3-with-residual pair, HIP-event timed (tile knob swept)."""
import math
import torch
from retr_amd import ops
from retr_amd._lib import call, ptr, load

DEV, bf = "cuda", torch.bfloat16


def timeit(fn, reps=50):
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
    for (N, H, W, C1, C2, Co, s) in [(16, 160, 160, 64, 64, 256, 1), (16, 80, 80, 128, 256, 512, 2),
                                     (16, 40, 40, 256, 512, 1024, 2),
                                     (16, 20, 20, 512, 1024, 2048, 2),
                                     (64, 28, 28, 512, 1024, 2048, 1)]:
        M = N * H * W
        H2, W2 = s * H, s * W
        x1 = torch.randn(M, C1, device=DEV).to(bf)
        x2 = torch.randn(N * H2 * W2, C2, device=DEV).to(bf)
        w1 = (torch.randn(Co, C1, device=DEV) / math.sqrt(C1)).to(bf)
        w2 = (torch.randn(Co, C2, device=DEV) / math.sqrt(C2)).to(bf)
        b = torch.randn(Co, device=DEV)
        wc = torch.cat([w1, w2], 1).contiguous()
        y = torch.empty(M, Co, dtype=bf, device=DEV)
        yd = torch.empty(M, Co, dtype=bf, device=DEV)
        st = ops._st()

        def fused():
            call("retr_conv1x1_fwd_cat", ops.dcode(bf), ptr(x1), C1, ptr(x2), C2, N, H, W, H2,
                 W2, s, ptr(wc), ptr(b), ptr(y), Co, 1, st)

        def unfused():
            call("retr_conv2d_fwd", ops.dcode(bf), ptr(x2), N, H2, W2, C2, ptr(w2), ptr(b), None,
                 ptr(yd), Co, 1, 1, s, 0, 1, 0, st)
            call("retr_conv2d_fwd", ops.dcode(bf), ptr(x1), N, H, W, C1, ptr(w1), ptr(b), ptr(yd),
                 ptr(y), Co, 1, 1, 1, 0, 1, 1, st)

        tu = timeit(unfused)
        byts = 2 * M * (C1 + C2 + Co)
        line = f"N{N} {H}x{W} [{C1}|{C2} s{s}]->{Co}: unfused {tu:7.1f} us"
        for knob in (0, 1, 2, 4, 6, 8, 9):
            load().retr_tune(6, knob)
            tf = timeit(fused)
            line += f" | fused t{knob} {tf:6.1f} us {byts / tf / 1e3:5.0f} GB/s"
        load().retr_tune(6, 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
