"""CPU restatement of the RefCOCO image pipeline (test infrastructure only: nothing under
retr_amd/ imports this module).

Follows the reference's per-item image path, ``RefCocoCaption.__getitem__``
(/root/reference/data_utils/refcoco.py:105-188) with the transforms of ``get_transforms``
(refcoco.py:14-46) and the helpers of /root/reference/data_utils/utils.py:

  crop_image_to_bb (utils.py:161-193)   bbox rounded with Python round(); target = image rows
                                        y..y+h, cols x..x+w; context = image with the box
                                        zeroed, context mask True inside the box
  pad_img_to_max   (utils.py:227-235)   PIL ImageOps.pad(size=(D, D), centering=(0.5, 0.5),
                                        color=0): no resampling (contain() keeps the size), the
                                        image pasted at round((D - side) * 0.5) (banker's
                                        rounding, Python round)
  pad_mask_to_max  (utils.py:238-252)   F.pad with True: floor(diff / 2) before, ceil after
  Resize(crop_size, BILINEAR)           PIL Image.resize BILINEAR on the uint8 image (two-pass
                                        antialiased triangle filter, 22-bit fixed point,
                                        horizontal pass first, uint8 between passes); on the
                                        bool mask tensor: antialiased bilinear in float, cast
                                        back to bool (nonzero -> True)
  ColorJitter(brightness=[0.5, 1.3], contrast=[0.8, 1.5], saturation=[0.2, 1.5]) (train)
                                        PIL ImageEnhance ops in a random order: blend(black, im,
                                        f), blend(mean-of-L grey, im, f), blend(L(im), im, f);
                                        blend in float32, truncated to uint8 (clipped outside
                                        [0, 1])
  ToTensor + Normalize(ImageNet mean / std)
  compute_position_features (utils.py:196-224)

The fixed-point resampler restates Pillow's libImaging/Resample.c (precompute_coeffs,
normalize_coeffs_8bpc, ImagingResampleHorizontal_8bpc / Vertical_8bpc); Pillow is importable in
this image, and tests/test_pipeline.py pins this restatement against it bit for bit.
"""
import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def round_half_even(x):
    """Python 3 round() (banker's rounding) -- what the reference's round(bb[i]) and Pillow's
    ImageOps.pad offsets use."""
    return int(round(x))


def crop_box(bb):
    """Integer (x, y, w, h) of refcoco bbox coordinates (utils.py:174)."""
    return tuple(round_half_even(v) for v in bb)


def pad_offsets_img(w, h):
    """(D, ox, oy) of pad_img_to_max for a w x h image (ImageOps.pad centering 0.5)."""
    D = max(w, h)
    ox = round_half_even((D - w) * 0.5) if w != D else 0
    oy = round_half_even((D - h) * 0.5) if w == D and h != D else 0
    return D, ox, oy


def pad_offsets_mask(w, h):
    """(D, ox, oy) of pad_mask_to_max for a mask of h rows x w cols: floor(diff / 2) before."""
    D = max(w, h)
    return D, (D - w) // 2, (D - h) // 2


def resample_coeffs(in_size, out_size):
    """Pillow precompute_coeffs (bilinear, support 1) + normalize_coeffs_8bpc.
    Returns (ksize, bounds [out][2] = (xmin, xcount), fixed-point coeffs [out][ksize] int32)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, ksize), dtype=np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        k = np.zeros(ksize, dtype=np.float64)
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w = 1.0 - t if t < 1.0 else 0.0
            k[x] = w
            ww += w
        for x in range(xmax):
            if ww != 0.0:
                k[x] /= ww
        for x in range(ksize):
            v = k[x] * (1 << PRECISION_BITS)
            kk[xx, x] = int(0.5 + v) if k[x] >= 0 else int(-0.5 + v)
        bounds[xx] = (xmin, xmax)
    return ksize, bounds, kk


def _clip8(acc):
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_u8(img, out_h, out_w):
    """Pillow Image.resize((out_w, out_h), BILINEAR) of an HxWx3 uint8 array."""
    h, w, _ = img.shape
    x = img
    if out_w != w:
        _, bx, kx = resample_coeffs(w, out_w)
        acc = np.full((h, out_w, 3), 1 << (PRECISION_BITS - 1), dtype=np.int64)
        for xx in range(out_w):
            x0, n = bx[xx]
            acc[:, xx, :] += np.einsum("hkc,k->hc", x[:, x0:x0 + n, :].astype(np.int64),
                                       kx[xx, :n].astype(np.int64))
        x = _clip8(acc)
    if out_h != h:
        _, by, ky = resample_coeffs(h, out_h)
        acc = np.full((out_h, x.shape[1], 3), 1 << (PRECISION_BITS - 1), dtype=np.int64)
        for yy in range(out_h):
            y0, n = by[yy]
            acc[yy] += np.einsum("kwc,k->wc", x[y0:y0 + n].astype(np.int64),
                                 ky[yy, :n].astype(np.int64))
        x = _clip8(acc)
    return x


def aa_window(in_size, out_size):
    """Nonzero-weight input window [lo, hi) per output index of the antialiased bilinear
    filter (torch _upsample_bilinear2d_aa / Pillow geometry)."""
    scale = in_size / out_size
    support = max(scale, 1.0)
    ss = 1.0 / support
    out = []
    for i in range(out_size):
        center = (i + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size)
        taps = [x for x in range(xmin, xmax) if abs((x - center + 0.5) * ss) < 1.0]
        out.append((taps[0], taps[-1] + 1) if taps else (xmin, xmin))
    return out


def resize_mask(mask, out_h, out_w):
    """torchvision Resize(BILINEAR) on a bool [H, W] mask: antialiased bilinear in float, cast to
    bool, i.e. True wherever a nonzero filter tap covers a True pixel."""
    h, w = mask.shape
    wy, wx = aa_window(h, out_h), aa_window(w, out_w)
    m = mask.astype(np.int32)
    cols = np.stack([m[:, a:b].max(axis=1) if b > a else np.zeros(h, np.int32)
                     for a, b in wx], axis=1)
    rows = np.stack([cols[a:b].max(axis=0) if b > a else np.zeros(out_w, np.int32)
                     for a, b in wy], axis=0)
    return rows.astype(bool)


def luma_u8(img):
    """Pillow RGB -> L: (R 19595 + G 38470 + B 7471 + 0x8000) >> 16."""
    i = img.astype(np.int64)
    return ((i[..., 0] * 19595 + i[..., 1] * 38470 + i[..., 2] * 7471 + 0x8000) >> 16) \
        .astype(np.uint8)


def blend_u8(degenerate, img, factor):
    """Pillow ImagingBlend(degenerate, img, alpha) with alpha a C float."""
    a = np.float32(factor)
    d = degenerate.astype(np.float32)
    t = d + a * (img.astype(np.float32) - d)
    if 0.0 <= a <= 1.0:
        return t.astype(np.int32).astype(np.uint8)
    return np.where(t <= 0, 0, np.where(t >= 255, 255, t.astype(np.int32))).astype(np.uint8)


def adjust(img, op, factor):
    """ColorJitter op 0 brightness / 1 contrast / 2 saturation (torchvision functional_pil ->
    ImageEnhance.Brightness / Contrast / Color)."""
    if op == 0:
        return blend_u8(np.zeros_like(img), img, factor)
    if op == 1:
        lum = luma_u8(img)
        mean = int(float(lum.astype(np.int64).sum()) / lum.size + 0.5)
        return blend_u8(np.full_like(img, mean), img, factor)
    if op == 2:
        return blend_u8(np.repeat(luma_u8(img)[..., None], 3, axis=2), img, factor)
    raise ValueError(op)


def normalize(img):
    """ToTensor + Normalize(ImageNet): [3, H, W] float32."""
    x = img.astype(np.float32).transpose(2, 0, 1) / np.float32(255.0)
    mean = np.array(IMAGENET_MEAN, dtype=np.float32)[:, None, None]
    std = np.array(IMAGENET_STD, dtype=np.float32)[:, None, None]
    return (x - mean) / std


def process(image, bb, size, jitter=None, context=False):
    """One encoder input of refcoco.py:131-178.  image: HxWx3 uint8; bb: (x, y, w, h) floats;
    jitter: None (val) or a list of (op, factor) in application order.
    Returns (uint8 [size, size, 3] after resize (+ jitter), float32 [3, size, size], bool mask)."""
    x, y, w, h = crop_box(bb)
    if context:
        region = image.copy()
        region[max(y, 0):max(y + h, 0), max(x, 0):max(x + w, 0)] = 0
        mask = np.zeros(image.shape[:2], dtype=bool)
        mask[max(y, 0):max(y + h, 0), max(x, 0):max(x + w, 0)] = True
    else:
        region = image[max(y, 0):max(y + h, 0), max(x, 0):max(x + w, 0)]
        mask = np.zeros(region.shape[:2], dtype=bool)
    rh, rw = region.shape[:2]
    D, ox, oy = pad_offsets_img(rw, rh)
    padded = np.zeros((D, D, 3), dtype=np.uint8)
    padded[oy:oy + rh, ox:ox + rw] = region
    Dm, mx, my = pad_offsets_mask(rw, rh)
    pm = np.ones((Dm, Dm), dtype=bool)
    pm[my:my + rh, mx:mx + rw] = mask
    out = resize_u8(padded, size, size)
    for op, f in (jitter or []):
        out = adjust(out, op, f)
    return out, normalize(out), resize_mask(pm, size, size)


def position_features(image_hw, bb):
    """compute_position_features (utils.py:196-224): [x1/iw, y1/ih, x2/iw, y2/ih, area]."""
    ih, iw = image_hw
    x, y, w, h = bb
    return np.array([x / iw, y / ih, (x + w) / iw, (y + h) / ih, (w * h) / (iw * ih)],
                    dtype=np.float32)
