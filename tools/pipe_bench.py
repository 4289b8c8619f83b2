"""Throughput of the RefCOCO encoder-input pipeline: the HIP path
(retr_amd.data_pipeline.RefCocoTransform, train mode: crop, pad, resize, ColorJitter, normalise,
mask) on batches of decoded COCO-sized images, against the reference's per-item CPU path
(Pillow crop / ImageOps.pad / resize / ImageEnhance + ToTensor / Normalize, as
data_utils/refcoco.py:131-178 runs it inside a DataLoader worker) on one host core.

    python tools/pipe_bench.py [--size 640] [--batch 16] [--reps 20]

Prints one JSON line: GPU images/s (host prep + upload + kernels, synchronised), the kernels
alone (HIP events), and the CPU images/s per core.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
from PIL import Image, ImageEnhance, ImageOps

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd import data_pipeline as dp  # noqa: E402


def _batch(n, seed):
    rng = np.random.default_rng(seed)
    imgs, bbs = [], []
    for _ in range(n):
        H, W = (480, 640) if rng.random() < 0.5 else (640, 480)
        imgs.append(rng.integers(0, 256, (H, W, 3), dtype=np.uint8))
        w, h = rng.uniform(40, W * 0.8), rng.uniform(40, H * 0.8)
        bbs.append((rng.uniform(0, W - w), rng.uniform(0, H - h), w, h))
    return imgs, bbs


def cpu_item(img, bb, S, jit):
    """The reference's per-item image path on the host (Pillow + numpy ToTensor/Normalize)."""
    x, y, w, h = (round(v) for v in bb)
    region = Image.fromarray(img[y:y + h, x:x + w])
    im = ImageOps.pad(region, (max(region.size),) * 2, centering=(0.5, 0.5), color=0)
    im = im.resize((S, S), Image.BILINEAR)
    for op, f in jit:
        im = {1: ImageEnhance.Brightness, 2: ImageEnhance.Contrast,
              3: ImageEnhance.Color}[op](im).enhance(f)
    a = np.asarray(im, dtype=np.float32).transpose(2, 0, 1) / 255.0
    return (a - np.array(dp.IMAGENET_MEAN, np.float32)[:, None, None]) / \
        np.array(dp.IMAGENET_STD, np.float32)[:, None, None]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    imgs, bbs = _batch(a.batch, 0)
    tf = dp.RefCocoTransform("train", a.size, generator=torch.Generator().manual_seed(0))
    for _ in range(3):
        tf(imgs, bbs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        tf(imgs, bbs)
    torch.cuda.synchronize()
    gpu = a.batch * a.reps / (time.perf_counter() - t0)
    # kernels alone: the same batch re-encoded between HIP events
    jit = [dp.jitter_params(torch.Generator().manual_seed(i)) for i in range(a.batch)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dp.encode(imgs, bbs, a.size, jit)
    ker = []
    for _ in range(5):
        e0.record()
        dp.encode(imgs, bbs, a.size, jit)
        e1.record()
        torch.cuda.synchronize()
        ker.append(e0.elapsed_time(e1))
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 5.0:
        cpu_item(imgs[n % a.batch], bbs[n % a.batch], a.size, jit[n % a.batch])
        n += 1
    cpu = n / (time.perf_counter() - t0)
    print(json.dumps({"metric": "RefCOCO encoder inputs/sec (train transforms)",
                      "size": a.size, "batch": a.batch,
                      "gpu_images_per_s": round(gpu, 1),
                      "gpu_ms_per_batch_incl_host_prep_and_upload": round(1e3 * a.batch / gpu, 3),
                      "gpu_stream_ms_per_batch_min": round(min(ker), 3),
                      "cpu_images_per_s_one_core": round(cpu, 1),
                      "cpu_sample": f"{n} items, Pillow {Image.__version__}"}))


if __name__ == "__main__":
    main()
