"""Deterministic mode (config.deterministic / retr_set_deterministic): fixed-order reductions
everywhere, so repeated runs on the same inputs are bitwise equal; and the (always
deterministic) DecoderEmbeddings backward against torch autograd
(models/transformer_modules.py:113-129)."""
import math

import pytest
import torch
import torch.nn.functional as F

from retr_amd import ops
from retr_amd import _lib
from retr_amd._lib import call, ptr
from retr_amd.models.utils import NestedTensor
from tests.helpers import make_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def det():
    ops.set_deterministic(True)
    yield
    ops.set_deterministic(False)


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def test_wgrad_and_bias_grad_bitwise_repeatable(det):
    """Shapes that split over K with fp32 atomics in the default mode."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 6400, 256, 256
    dy = torch.randn(M, N, generator=g).to(DEV).bfloat16()
    x = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    outs = []
    for _ in range(2):
        dw = torch.zeros(N, K, device=DEV)
        db = torch.zeros(N, device=DEV)
        ops.k_linear_wgrad(dy, x, dw, db)
        db2 = torch.zeros(N, device=DEV)
        ops.k_bias_grad(dy, db2)
        outs.append((dw, db, db2))
    ref_w = dy.float().t() @ x.float()
    ref_b = dy.float().sum(0)
    assert _rel(outs[0][0], ref_w) < 1e-5 and _rel(outs[0][1], ref_b) < 1e-5
    assert _rel(outs[0][2], ref_b) < 1e-5
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    # conv weight gradient (pixel reduction of 25600)
    Nb, H, C, Co = 8, 40, 256, 256
    gn = torch.randn(Nb, H, H, Co, generator=g).to(DEV).bfloat16()
    xn = torch.randn(Nb, H, H, C, generator=g).to(DEV).bfloat16()
    splits = _lib.load().retr_conv2d_wgrad_splits(ops.dcode(torch.bfloat16), Nb, H, H, C, Co,
                                                  3, 3, 1, 1, 1)
    assert splits > 1            # the reduction is sliced: the slabs are added in order
    wss = []
    for _ in range(2):
        ws = torch.empty(splits, Co, 9 * C, device=DEV)
        call("retr_conv2d_wgrad", ops.dcode(torch.bfloat16), ptr(gn), ptr(xn), Nb, H, H, C,
             ptr(ws), Co, 3, 3, 1, 1, 1, ops._st())
        grad = torch.empty(Co, C, 3, 3, device=DEV)
        call("retr_conv_wgrad_unpack", ptr(ws), None, ptr(grad), Co, C, C, 3, 3, 0, splits,
             ops._st())
        wss.append(grad)
    assert torch.equal(wss[0], wss[1])
    ref = torch.nn.grad.conv2d_weight(xn.permute(0, 3, 1, 2).float().cpu(), (Co, C, 3, 3),
                                      gn.permute(0, 3, 1, 2).float().cpu(), padding=1)
    assert _rel(wss[0].cpu(), ref) < 1e-5


@pytest.mark.parametrize("padding_idx", [0, None])
def test_embed_ln_backward_matches_autograd(padding_idx):
    """word/position/LayerNorm gradients of the fused DecoderEmbeddings backward, with repeated
    tokens and the padding row (no gradient to padding_idx, nn.Embedding semantics)."""
    g = torch.Generator().manual_seed(7)
    B, T, C, V = 8, 32, 256, 50
    caps = torch.randint(0, V, (B, T), generator=g)
    caps[:, -5:] = 0                                   # padding tokens
    word = torch.randn(V, C, generator=g)
    posw = torch.randn(T + 3, C, generator=g)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    dy = torch.randn(B * T, C, generator=g)
    ps = [t.to(DEV).requires_grad_(True) for t in (word, posw, gamma, beta)]
    y = ops._EmbedLN.apply(caps.to(DEV), *ps, 1e-12, 0.0, padding_idx, False)
    y.backward(dy.to(DEV))
    rs = [t.clone().requires_grad_(True) for t in (word, posw, gamma, beta)]
    e = rs[0][caps] + rs[1][:T].unsqueeze(0)
    ref = F.layer_norm(e, (C,), rs[2], rs[3], 1e-12).reshape(B * T, C)
    ref.backward(dy)
    gw = rs[0].grad.clone()
    if padding_idx is not None:
        gw[padding_idx] = 0
    assert _rel(y.detach().cpu(), ref.detach()) < 1e-6
    for got, want in zip([p.grad for p in ps], [gw, rs[1].grad, rs[2].grad, rs[3].grad]):
        assert _rel(got.cpu(), want) < 1e-5
    if padding_idx is not None:
        assert torch.count_nonzero(ps[0].grad[padding_idx]) == 0
    # bitwise repeatable
    first = [p.grad.clone() for p in ps]
    for p in ps:
        p.grad = None
    ops._EmbedLN.apply(caps.to(DEV), *ps, 1e-12, 0.0, padding_idx, False).backward(dy.to(DEV))
    for a, p in zip(first, ps):
        assert torch.equal(a, p.grad)


def test_bf16_training_steps_bitwise_repeatable(det):
    """Two identical bf16 models, two reference training steps each (forward, CE, backward,
    fused clip + AdamW): every parameter bitwise equal."""
    from bench import build, make_optimizer
    from retr_amd.engine import train_step
    from retr_amd.synthetic import synthetic_captions, synthetic_images
    cfg = make_config(backbone="ResNet50", dilation=True, hidden=64, layers=(2, 2), vocab=1000,
                      max_pos=16, ffn=128, dtype="bf16")
    img, mask = synthetic_images(4, 96, seed=5, pad_band=True)
    caps, cm = synthetic_captions(4, cfg.max_position_embeddings, cfg.vocab_size, seed=6)
    samples = (NestedTensor(img.to(DEV), mask.to(DEV)),)
    finals = []
    for _ in range(2):
        model, crit = build(cfg, DEV)
        model.train()
        opt = make_optimizer(model, cfg, fused=True)
        for _ in range(2):
            loss = train_step(model, crit, samples, caps.to(DEV), cm.to(DEV), opt, 0.1)
        assert math.isfinite(loss.item())
        finals.append([p.detach().clone() for p in model.parameters()])
    for a, b in zip(*finals):
        assert torch.equal(a, b)
