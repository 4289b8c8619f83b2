"""Decode-only driver for profiling (rocprofv3 --kernel-trace --stats -- python tools/decode_prof.py):
cfg5 (ResNet-50 dilation 224x224, 6/6 d256, bf16), batch 64, greedy (and beam with --beam K),
captured step graphs; prints ms per batch and per step."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import build, cfg5  # noqa: E402
from retr_amd.eval_utils.decode import IncrementalBeam, greedy  # noqa: E402
from retr_amd.models.utils import NestedTensor  # noqa: E402
from retr_amd.synthetic import synthetic_images  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--beam", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--fold", type=int, default=None,
                    help="1 / 0: eval_utils.decode.DEC_FOLD_ROWS (default: the module's)")
    ap.add_argument("--ffn-ln", type=int, default=None,
                    help="1 / 0: eval_utils.decode.DEC_FFN_LN (default: the module's)")
    ap.add_argument("--fold-max-rows", type=int, default=None,
                    help="eval_utils.decode.DEC_FOLD_MAX_ROWS (default: the module's)")
    ap.add_argument("--fp32", action="store_true", help="cfg5 in fp32 parity mode")
    ap.add_argument("--f32-fused", type=int, default=None,
                    help="1 / 0: eval_utils.decode.DEC_F32_FUSED (default: the module's)")
    ap.add_argument("--hb128-rows", type=int, default=None,
                    help="eval_utils.decode.DEC_FFN_HB128_ROWS (default: the module's)")
    ap.add_argument("--select-embed", type=int, default=None,
                    help="1 / 0: eval_utils.decode.DEC_SELECT_EMBED (default: the module's)")
    ap.add_argument("--head-skinny", type=int, default=0,
                    help="1 / 2: eval_utils.decode.DEC_HEAD_SKINNY on / off (0: the module's)")
    ap.add_argument("--rows-per-block", type=int, default=None,
                    help="eval_utils.decode.DEC_ROWS_PER_BLOCK (default: automatic)")
    ap.add_argument("--block-per-row", action="store_true",
                    help="the round-4 attention sub-layers (eval_utils.decode.DEC_HEADS = False)")
    a = ap.parse_args()
    from retr_amd.eval_utils import decode as dec
    dec.DEC_HEADS = not a.block_per_row
    if a.ffn_ln is not None:
        dec.DEC_FFN_LN = bool(a.ffn_ln)
    if a.fold is not None:
        dec.DEC_FOLD_ROWS = bool(a.fold)
    dec.DEC_ROWS_PER_BLOCK = a.rows_per_block
    if a.hb128_rows is not None:
        dec.DEC_FFN_HB128_ROWS = a.hb128_rows
    if a.select_embed is not None:
        dec.DEC_SELECT_EMBED = bool(a.select_embed)
    if a.head_skinny:
        dec.DEC_HEAD_SKINNY = a.head_skinny == 1
    if a.f32_fused is not None:
        dec.DEC_F32_FUSED = bool(a.f32_fused)
    if a.fold_max_rows is not None:
        dec.DEC_FOLD_MAX_ROWS = a.fold_max_rows
    model, _ = build(cfg5("fp32") if a.fp32 else cfg5(), "cuda")
    model.eval()
    img, mask = synthetic_images(a.batch, 224, seed=3000)
    samples = [NestedTensor(img.cuda(), mask.cuda())]
    T = 128
    if a.beam > 1:
        bm = IncrementalBeam(model, a.beam)
        fn = lambda: bm(samples, T, 101, 102)  # noqa: E731
    else:
        fn = lambda: greedy(samples, model, max_len=T, bos_token=101, eos_token=102)  # noqa: E731
    ids = fn()
    torch.cuda.synchronize()
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ids = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = int((ids != 0).sum(1).max().item())
        print(f"beam {a.beam}: {dt * 1e3:.2f} ms/batch, {a.batch / dt:.1f} refs/s, "
              f"{dt * 1e3 / max(1, steps - 1):.3f} ms/step over {steps} tokens", flush=True)


if __name__ == "__main__":
    main()
