"""RefCOCO input pipeline: the CPU restatement (oracle/pipeline.py) pinned
against Pillow and torch -- the libraries the reference's transforms call -- and the HIP pipeline
(retr_amd/data_pipeline.py, csrc/pipeline.hip) against the restatement, bit for bit.

Reference path: data_utils/refcoco.py:131-178 (crop_image_to_bb, pad_img_to_max,
pad_mask_to_max, Resize, ColorJitter, ToTensor, Normalize) with data_utils/utils.py:161-252."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from PIL import Image, ImageEnhance, ImageOps

from oracle import pipeline as P

# (image H, W, bbox x, y, w, h, output size): down- and up-scaling, odd pad differences
# (banker's rounding of ImageOps.pad vs floor of pad_mask_to_max), tall / wide / square crops,
# a box at the image edge and one that overhangs it
CASES = [
    (480, 640, (100.4, 50.6, 300.2, 200.5), 224),
    (300, 200, (10.5, 20.5, 33.0, 91.0), 224),
    (500, 500, (0.0, 0.0, 500.0, 500.0), 224),
    (60, 80, (3.5, 4.5, 51.0, 40.0), 640),
    (427, 640, (590.2, 300.7, 49.6, 126.3), 224),
    (375, 500, (12.0, 7.0, 21.0, 14.0), 224),
    (640, 480, (0.0, 100.0, 480.0, 300.0), 640),
]
JIT = [[(1, 0.7), (2, 1.4), (3, 0.3)], [(3, 1.45), (1, 1.2), (2, 0.85)], [(2, 1.1)], []]


def _image(H, W, seed):
    rng = np.random.default_rng(seed)
    # smooth + noise so resampling and the luma mean are non-trivial
    yy, xx = np.mgrid[0:H, 0:W]
    base = np.stack([(xx * 255 // max(W - 1, 1)), (yy * 255 // max(H - 1, 1)),
                     ((xx + yy) * 7) % 256], axis=-1)
    return np.clip(base + rng.integers(-40, 41, base.shape), 0, 255).astype(np.uint8)


def _pil_target(img, bb, S):
    x, y, w, h = P.crop_box(bb)
    region = Image.fromarray(img[y:y + h, x:x + w])
    padded = ImageOps.pad(region, (max(region.size),) * 2, centering=(0.5, 0.5), color=0)
    return padded.resize((S, S), Image.BILINEAR)


@pytest.mark.parametrize("case", CASES)
def test_oracle_resize_matches_pillow(case):
    H, W, bb, S = case
    img = _image(H, W, sum(map(int, bb)))
    u8, _, _ = P.process(img, bb, S)
    assert np.array_equal(np.asarray(_pil_target(img, bb, S)), u8)


@pytest.mark.parametrize("op,factor", [(1, 0.5), (1, 0.93), (1, 1.3), (2, 0.8), (2, 1.27),
                                       (2, 1.5), (3, 0.2), (3, 0.66), (3, 1.5)])
def test_oracle_jitter_matches_pillow(op, factor):
    pil = _pil_target(_image(300, 400, 7), (50.2, 30.1, 250.5, 199.9), 224)
    enh = {1: ImageEnhance.Brightness, 2: ImageEnhance.Contrast, 3: ImageEnhance.Color}[op]
    ref = np.asarray(enh(pil).enhance(factor))
    assert np.array_equal(ref, P.adjust(np.asarray(pil), op - 1, factor))


@pytest.mark.parametrize("h,w,S", [(200, 300, 224), (33, 91, 224), (91, 33, 640),
                                   (700, 640, 224), (224, 224, 224)])
def test_oracle_mask_resize_matches_torch(h, w, S):
    D, mx, my = P.pad_offsets_mask(w, h)
    pm = np.ones((D, D), bool)
    pm[my:my + h, mx:mx + w] = False
    ref = F.interpolate(torch.from_numpy(pm).float()[None, None], size=(S, S), mode="bilinear",
                        align_corners=False, antialias=True)[0, 0] != 0
    assert np.array_equal(ref.numpy(), P.resize_mask(pm, S, S))


def test_host_tables_match_oracle():
    from retr_amd import data_pipeline as dp
    for D, S in [(640, 224), (33, 224), (224, 224), (91, 640), (1000, 224), (7, 3)]:
        k1, b1, kk1 = dp._coeffs(D, S)
        k2, b2, kk2 = P.resample_coeffs(D, S)
        assert k1 == k2 and np.array_equal(b1, b2) and np.array_equal(kk1, kk2)
        assert np.array_equal(dp._windows(D, S), np.array(P.aa_window(D, S)))


def test_jitter_params_follow_torchvision_draw_order():
    from retr_amd import data_pipeline as dp
    g1, g2 = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    got = dp.jitter_params(g1)
    perm = torch.randperm(4, generator=g2).tolist()
    fs = [float(torch.empty(1).uniform_(lo, hi, generator=g2))
          for lo, hi in ((0.5, 1.3), (0.8, 1.5), (0.2, 1.5))]
    assert got == [(i + 1, fs[i]) for i in perm if i != 3]
    assert all(0.2 <= f <= 1.5 for _, f in got)


@pytest.mark.gpu
@pytest.mark.parametrize("context", [False, True])
def test_gpu_pipeline_bit_exact(context):
    from retr_amd import data_pipeline as dp
    imgs = [_image(H, W, i) for i, (H, W, _, _) in enumerate(CASES)]
    for S in (224, 640):
        idx = [i for i, c in enumerate(CASES)]
        bbs = [CASES[i][2] for i in idx]
        jit = [JIT[i % len(JIT)] for i in idx]
        out, mask, u8 = dp.encode(imgs, bbs, S, jit, context=context, want_u8=True)
        torch.cuda.synchronize()
        for i in idx:
            ref_u8, ref_f, ref_m = P.process(imgs[i], bbs[i], S,
                                             [(op - 1, f) for op, f in jit[i]], context=context)
            assert np.array_equal(u8[i].cpu().numpy(), ref_u8), (S, i)
            assert np.array_equal(out[i].cpu().numpy(), ref_f), (S, i)
            assert np.array_equal(mask[i].cpu().numpy(), ref_m), (S, i)


@pytest.mark.gpu
def test_gpu_transform_api():
    from retr_amd import data_pipeline as dp
    imgs = [_image(H, W, i) for i, (H, W, _, _) in enumerate(CASES)]
    bbs = [c[2] for c in CASES]
    tf = dp.RefCocoTransform("val", 224, return_global_context=True,
                             return_location_features=True)
    t_img, t_mask, g_img, g_mask, loc = tf(imgs, bbs)
    assert t_img.shape == (len(imgs), 3, 224, 224) and t_img.dtype == torch.float32
    assert t_mask.dtype == torch.bool and g_mask.shape == (len(imgs), 224, 224)
    ref = np.stack([P.position_features(im.shape[:2], bb) for im, bb in zip(imgs, bbs)])
    assert np.allclose(loc.cpu().numpy(), ref, rtol=0, atol=0)
    for i in range(len(imgs)):
        _, f, m = P.process(imgs[i], bbs[i], 224, context=True)
        assert np.array_equal(g_img[i].cpu().numpy(), f) and np.array_equal(g_mask[i].cpu().numpy(), m)
    # train mode draws jitter from the generator: same seed -> same batch
    a = dp.RefCocoTransform("train", 224, generator=torch.Generator().manual_seed(5))(imgs, bbs)
    b = dp.RefCocoTransform("train", 224, generator=torch.Generator().manual_seed(5))(imgs, bbs)
    assert torch.equal(a[0], b[0]) and not torch.equal(a[0], t_img)
    with pytest.raises(NotImplementedError):
        dp.RefCocoTransform("bogus")
