"""RefCOCO encoder inputs built on the GPU.

Mirrors the image half of ``RefCocoCaption.__getitem__`` (data_utils/refcoco.py:131-178) with
``get_transforms`` (refcoco.py:14-46) for a whole batch at once:

    tf = RefCocoTransform("train", size=224, return_global_context=False,
                          return_location_features=False)
    t_img, t_mask, *rest = tf(images, bbs)          # images: HxWx3 uint8 arrays (decoded RGB)

returns stacked tensors on the current device in the order the reference builds
``encoder_input`` (refcoco.py:153-178): target image [B, 3, S, S] fp32, target mask [B, S, S]
bool, then (global context) image + mask, then (location) position features [B, 5].

What stays on the host: JPEG decoding (PIL, as the reference), the bbox arithmetic, Pillow's
double-precision resampling coefficients (computed once per (D, S) and cached) and the
ColorJitter draws (torchvision ColorJitter.get_params order: randperm(4), then the brightness,
contrast, saturation factors).  Everything per pixel -- crop / context masking, pad-to-square,
antialiased bilinear resize, jitter blends, ToTensor + Normalize, mask resize -- runs in
``csrc/pipeline.hip`` after one upload of the raw uint8 pixels, bit-exact with Pillow
(tests/test_pipeline.py).  Bounding boxes are clamped to the image (the reference's numpy
slicing would wrap a negative start).
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr
from .ops import _st

PRECISION_BITS = 22
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
JITTER = {"brightness": (0.5, 1.3), "contrast": (0.8, 1.5), "saturation": (0.2, 1.5)}

_COEF = {}
_WIN = {}


def _coeffs(in_size, out_size):
    """Pillow precompute_coeffs (bilinear) + normalize_coeffs_8bpc, vectorised over outputs with
    the C loop's summation order: (ksize, int32 [out][2] bounds, int32 [out][ksize])."""
    key = (in_size, out_size)
    hit = _COEF.get(key)
    if hit is not None:
        return hit
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    center = (np.arange(out_size, dtype=np.float64) + 0.5) * scale
    xmin = np.maximum(np.trunc(center - support + 0.5).astype(np.int64), 0)
    xmax = np.minimum(np.trunc(center + support + 0.5).astype(np.int64), in_size) - xmin
    ss = 1.0 / filterscale
    k = np.zeros((out_size, ksize), dtype=np.float64)
    ww = np.zeros(out_size, dtype=np.float64)
    for x in range(ksize):
        t = np.abs((x + xmin - center + 0.5) * ss)
        w = np.where((x < xmax) & (t < 1.0), 1.0 - t, 0.0)
        k[:, x] = w
        ww = ww + w
    nz = ww != 0.0
    k[nz] = k[nz] / ww[nz, None]
    v = k * float(1 << PRECISION_BITS)
    kk = np.where(k >= 0, np.trunc(0.5 + v), np.trunc(-0.5 + v)).astype(np.int32)
    bounds = np.stack([xmin, xmax], axis=1).astype(np.int32)
    out = (ksize, bounds, kk)
    _COEF[key] = out
    return out


def _windows(in_size, out_size):
    """Nonzero-tap window [lo, hi) per output of the antialiased bilinear mask resize
    (torchvision Resize on the bool mask tensor: aa-bilinear, cast back to bool)."""
    key = (in_size, out_size)
    hit = _WIN.get(key)
    if hit is not None:
        return hit
    scale = in_size / out_size
    support = max(scale, 1.0)
    ss = 1.0 / support
    center = (np.arange(out_size, dtype=np.float64) + 0.5) * scale
    xmin = np.maximum(np.trunc(center - support + 0.5).astype(np.int64), 0)
    xmax = np.minimum(np.trunc(center + support + 0.5).astype(np.int64), in_size)
    lo = np.full(out_size, -1, dtype=np.int64)
    hi = np.full(out_size, -1, dtype=np.int64)
    width = int(xmax.max() - xmin.min()) + 1 if out_size else 0
    for j in range(width + 1):
        x = xmin + j
        ok = (x < xmax) & (np.abs((x - center + 0.5) * ss) < 1.0)
        lo = np.where(ok & (lo < 0), x, lo)
        hi = np.where(ok, x + 1, hi)
    empty = lo < 0
    lo = np.where(empty, xmin, lo)
    hi = np.where(empty, xmin, hi)
    out = np.stack([lo, hi], axis=1).astype(np.int32)
    _WIN[key] = out
    return out


def round_half_even(v):
    return int(round(v))


def jitter_params(generator=None):
    """torchvision ColorJitter.get_params for (brightness, contrast, saturation, hue=None):
    [(op, factor)] in application order, op 1 brightness / 2 contrast / 3 saturation."""
    perm = torch.randperm(4, generator=generator).tolist()
    fs = [float(torch.empty(1).uniform_(lo, hi, generator=generator))
          for lo, hi in JITTER.values()]
    return [(i + 1, fs[i]) for i in perm if i != 3]


class _Item(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_longlong), ("tmp_off", ctypes.c_longlong),
                ("H", ctypes.c_int), ("W", ctypes.c_int), ("x0", ctypes.c_int),
                ("y0", ctypes.c_int), ("rw", ctypes.c_int), ("rh", ctypes.c_int),
                ("bx", ctypes.c_int), ("by", ctypes.c_int), ("bw", ctypes.c_int),
                ("bh", ctypes.c_int), ("D", ctypes.c_int), ("ox", ctypes.c_int),
                ("oy", ctypes.c_int), ("mx", ctypes.c_int), ("my", ctypes.c_int),
                ("coef_off", ctypes.c_int), ("ksize", ctypes.c_int), ("win_off", ctypes.c_int),
                ("ops", ctypes.c_int), ("f", ctypes.c_float * 3), ("pad_", ctypes.c_int * 2)]


def encode(images, bbs, size, jitters=None, context=False, device=None, want_u8=False):
    """Run the pipeline on a batch.  images: HxWx3 uint8 arrays; bbs: (x, y, w, h);
    jitters: per item None or [(op, factor)].  Returns (fp32 [B, 3, S, S], bool [B, S, S]) and,
    with want_u8, the uint8 [B, S, S, 3] image before normalisation."""
    dev = torch.device(device) if device is not None else torch.device("cuda")
    _lib.require_device(torch.empty(0, device=dev))
    n, S = len(images), int(size)
    items = (_Item * max(n, 1))()
    coef_parts, win_parts, src_parts = [], [], []
    coef_len = win_len = src_len = tmp_len = 0
    max_d = 1
    for i, (img, bb) in enumerate(zip(images, bbs)):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError(f"item {i}: expected an HxWx3 uint8 RGB image, got {img.shape}")
        H, W = img.shape[:2]
        x, y, w, h = (round_half_even(v) for v in bb)
        cx0, cy0 = min(max(x, 0), W), min(max(y, 0), H)
        cx1, cy1 = min(max(x + w, 0), W), min(max(y + h, 0), H)
        it = items[i]
        it.H, it.W = H, W
        if context:        # crop_image_to_bb(return_context=True): whole image, box zeroed
            it.x0, it.y0, it.rw, it.rh = 0, 0, W, H
            it.bx, it.by, it.bw, it.bh = cx0, cy0, cx1 - cx0, cy1 - cy0
        else:
            it.x0, it.y0, it.rw, it.rh = cx0, cy0, cx1 - cx0, cy1 - cy0
            it.bx = it.by = it.bw = it.bh = 0
        rw, rh = it.rw, it.rh
        if rw <= 0 or rh <= 0:
            raise ValueError(f"item {i}: empty crop for bbox {bb} in a {W}x{H} image")
        D = max(rw, rh)
        it.D = D
        it.ox = round_half_even((D - rw) * 0.5) if rw != D else 0
        it.oy = round_half_even((D - rh) * 0.5) if rw == D and rh != D else 0
        it.mx, it.my = (D - rw) // 2, (D - rh) // 2
        ksize, bounds, kk = _coeffs(D, S)
        it.coef_off, it.ksize = coef_len, ksize
        coef_parts.append(np.concatenate([bounds.reshape(-1), kk.reshape(-1)]))
        coef_len += coef_parts[-1].size
        it.win_off = win_len
        win_parts.append(_windows(D, S).reshape(-1))
        win_len += win_parts[-1].size
        it.src_off = src_len
        src_parts.append(img.reshape(-1))
        src_len += img.size
        it.tmp_off = tmp_len
        tmp_len += D * S * 3
        max_d = max(max_d, D)
        ops = 0
        for slot, (op, f) in enumerate(jitters[i] if jitters and jitters[i] else []):
            ops |= int(op) << (4 * slot)
            it.f[slot] = float(f)
        it.ops = ops
    out = torch.empty(n, 3, S, S, dtype=torch.float32, device=dev)
    mask = torch.empty(n, S, S, dtype=torch.bool, device=dev)
    u8 = torch.empty(n, S, S, 3, dtype=torch.uint8, device=dev)
    if n == 0:
        return (out, mask, u8) if want_u8 else (out, mask)
    src = torch.from_numpy(np.concatenate(src_parts)).pin_memory().to(dev, non_blocking=True)
    coef = torch.from_numpy(np.concatenate(coef_parts).astype(np.int32)).to(dev)
    win = torch.from_numpy(np.concatenate(win_parts).astype(np.int32)).to(dev)
    desc = torch.frombuffer(bytearray(bytes(items)[: n * ctypes.sizeof(_Item)]),
                            dtype=torch.uint8).to(dev)
    tmp = torch.empty(tmp_len, dtype=torch.uint8, device=dev)
    mean = (ctypes.c_float * 3)(*IMAGENET_MEAN)
    std = (ctypes.c_float * 3)(*IMAGENET_STD)
    call("retr_pipe_run", ptr(src), ptr(desc), n, ptr(coef), ptr(win), ptr(tmp), max_d, ptr(u8),
         ptr(out), ptr(mask), S, ctypes.cast(mean, ctypes.c_void_p),
         ctypes.cast(std, ctypes.c_void_p), _st())
    # the host buffers above must outlive the copies; the stream orders everything after them
    torch.cuda.current_stream(dev).synchronize()
    return (out, mask, u8) if want_u8 else (out, mask)


def position_features(images, bbs, device=None):
    """compute_position_features (data_utils/utils.py:196-224) per item -> [B, 5] fp32."""
    rows = []
    for img, (x, y, w, h) in zip(images, bbs):
        ih, iw = np.asarray(img).shape[:2]
        rows.append([x / iw, y / ih, (x + w) / iw, (y + h) / ih, (w * h) / (iw * ih)])
    return torch.tensor(rows, dtype=torch.float32, device=device or "cuda")


class RefCocoTransform:
    """Batched GPU counterpart of ``get_transforms(mode, config)`` + the image steps of
    ``RefCocoCaption.__getitem__``: ``mode`` 'train' (ColorJitter) or 'val'; ``size`` the
    weights' crop size (224 for the torchvision ResNet defaults, refcoco.py:17-25)."""

    def __init__(self, mode, size=224, return_global_context=False,
                 return_location_features=False, generator=None):
        if mode.lower() in ("training", "train"):
            self.train = True
        elif mode.lower() in ("val", "validation", "test", "eval"):
            self.train = False
        else:
            raise NotImplementedError(f"transforms mode {mode} is not implemented")
        self.size = size
        self.return_global_context = return_global_context
        self.return_location_features = return_location_features
        self.generator = generator

    def __call__(self, images, bbs, device=None):
        jit = [jitter_params(self.generator) for _ in images] if self.train else None
        t_img, t_mask = encode(images, bbs, self.size, jit, context=False, device=device)
        out = [t_img, t_mask]
        if self.return_global_context:
            gjit = [jitter_params(self.generator) for _ in images] if self.train else None
            out += list(encode(images, bbs, self.size, gjit, context=True, device=device))
        if self.return_location_features:
            out.append(position_features(images, bbs, device=t_img.device))
        return tuple(out)
