"""Per-kernel numerics of libretr_hip.so against plain PyTorch fp32 references (GPU box)."""
import math
import numpy as np

import pytest
import torch
import torch.nn.functional as F

from retr_amd import _lib, ops, resnet
from retr_amd._lib import call, ptr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (200, 96, 136), (2048, 256, 256),
                                   (4100, 520, 72), (37, 30522, 64),
                                   (6400, 2048, 256), (5000, 1800, 264), (5000, 264, 1800)])
def test_linear_fwd_dgrad_wgrad(dtype, tol, M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = torch.randn(N, K, generator=g).to(DEV) / math.sqrt(K)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    xc, wc = x.to(dtype), w.to(dtype)
    y = torch.empty(M, N, device=DEV)
    ops.k_linear_fwd(xc, wc, b, y, relu=1, res=res)
    ref = torch.relu(xc.float() @ wc.float().t() + b) + res
    assert rel_err(y, ref) < tol
    # dgrad with gate and addend
    Np = (N + 7) // 8 * 8
    dy = torch.zeros(M, Np, device=DEV)
    dy[:, :N] = torch.randn(M, N, generator=g).to(DEV)
    dyc = dy.to(dtype)
    wpad = torch.zeros(Np, K, device=DEV, dtype=dtype)
    wpad[:N] = wc
    gate = torch.randn(M, K, generator=g).to(DEV).to(dtype)
    add = torch.randn(M, K, generator=g).to(DEV)
    dx = torch.empty(M, K, device=DEV)
    ops.k_linear_dgrad(dyc, wpad.t().contiguous(), dx, addend=add, gate=gate)
    ref = (dyc.float() @ wpad.float() + add) * (gate.float() > 0)
    assert rel_err(dx, ref) < tol
    dw = torch.zeros(Np, K, device=DEV)
    ops.k_linear_wgrad(dyc, xc, dw)
    ref = dyc.float().t() @ xc.float()
    assert rel_err(dw, ref) < tol
    db = torch.zeros(Np, device=DEV)
    ops.k_bias_grad(dyc, db)
    assert rel_err(db, dyc.float().sum(0)) < tol
    # fused bias gradient + accumulate mode
    dw2 = torch.ones(Np, K, device=DEV)
    db2 = torch.ones(Np, device=DEV)
    ops.k_linear_wgrad(dyc, xc, dw2, db2, accumulate=True)
    assert rel_err(dw2, ref + 1) < tol
    assert rel_err(db2, dyc.float().sum(0) + 1) < tol
    dw3 = torch.full((Np, K), float("nan"), device=DEV)
    db3 = torch.full((Np,), float("nan"), device=DEV)
    ops.k_linear_wgrad(dyc, xc, dw3, db3)           # overwrite mode: no pre-zeroing needed
    assert rel_err(dw3, ref) < tol and rel_err(db3, dyc.float().sum(0)) < tol
    # exactly N output rows from the column-padded dy (the MLP head's vocab gradient)
    dw4 = torch.zeros(N, K, device=DEV)
    db4 = torch.zeros(N, device=DEV)
    ops.k_linear_wgrad(dyc, xc, dw4, db4, accumulate=True)
    assert rel_err(dw4, ref[:N]) < tol and rel_err(db4, dyc.float().sum(0)[:N]) < tol


# grouped launches (csrc/linear_group.hip): shapes of one attention / FFN block, ragged edges
GROUPS = {
    "enc_attn": [(6400, 512, 256), (6400, 256, 256), (6400, 256, 256)],
    "dec_cross": [(2048, 256, 256), (6400, 256, 256), (6400, 256, 256), (2048, 256, 256)],
    "ffn": [(6400, 2048, 256), (6400, 256, 2048)],
    "dec_ffn": [(2048, 2048, 256), (2048, 256, 2048)],
    "small_ragged": [(100, 64, 64), (37, 136, 72), (513, 264, 128)],
}


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("name", list(GROUPS))
def test_linear_groups(dtype, tol, name):
    shapes = GROUPS[name]
    g = torch.Generator(device="cpu").manual_seed(len(name))
    rnd = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(DEV)  # noqa: E731
    # forward: y = relu?(x W^T + b) (+ res), alternating variants, all bf16 / fp32 outputs
    for y_f32 in (False, True):
        items, refs = [], []
        for i, (M, N, K) in enumerate(shapes):
            x, w, b = rnd(M, K).to(dtype), rnd(N, K, sc=K ** -0.5).to(dtype), rnd(N)
            relu, res = i % 2, (rnd(M, N) if (y_f32 and i % 2 == 0) else None)
            y = torch.empty(M, N, device=DEV, dtype=torch.float32 if y_f32 else dtype)
            items.append((x, w, b, y, relu, res))
            r = x.float() @ w.float().t() + b
            r = torch.relu(r) if relu else r
            refs.append(r + res if res is not None else r)
        ops.k_linear_fwd_group(items)
        for it, r in zip(items, refs):
            assert rel_err(it[3].float(), r) < tol
    # data gradients: dx = gate(dy W [+ addend]), W read transposed (_TView) or W^T copies
    for view in (True, False):
        items, refs = [], []
        for i, (M, N, K) in enumerate(shapes):
            dy, w = rnd(M, N).to(dtype), rnd(N, K, sc=N ** -0.5).to(dtype)
            gate = rnd(M, K).to(dtype) if i % 2 else None
            add = rnd(M, K) if i == 0 else None
            dx = torch.empty(M, K, device=DEV)
            wt = ops._TView(w) if view else w.t().contiguous()
            items.append((dy, wt, dx, add, gate) if add is not None or gate is not None
                         else (dy, wt, dx))
            r = dy.float() @ w.float()
            r = r + add if add is not None else r
            refs.append(r * (gate.float() > 0) if gate is not None else r)
        # addend must be uniformly fp32 or absent within a group: split the first one off
        ops.k_linear_dgrad_group(items[:1])
        ops.k_linear_dgrad_group([(it[0], it[1], it[2], None, it[4]) if len(it) > 3 else it
                                  for it in items[1:]])
        for it, r in zip(items, refs):
            assert rel_err(it[2], r) < tol
    # weight + bias gradients, accumulate and overwrite, twice: bit-identical (ordered sums)
    for acc in (True, False):
        items, refs = [], []
        for i, (M, N, K) in enumerate(shapes):
            dy, x = rnd(M, N).to(dtype), rnd(M, K).to(dtype)
            dw = torch.ones(N, K, device=DEV) if acc else torch.full((N, K), float("nan"),
                                                                     device=DEV)
            db = (torch.ones(N, device=DEV) if acc else torch.full((N,), float("nan"),
                                                                   device=DEV)) \
                if i != 1 else None
            items.append((dy, x, dw, db, acc))
            refs.append((dy.float().t() @ x.float() + acc, dy.float().sum(0) + acc))
        ops.k_linear_wgrad_group(items)
        first = [(it[2].clone(), None if it[3] is None else it[3].clone()) for it in items]
        for it, (rw, rb) in zip(items, refs):
            assert rel_err(it[2], rw) < tol
            if it[3] is not None:
                assert rel_err(it[3], rb) < tol
        if not acc and dtype == torch.bfloat16:   # (fp32 runs the single-GEMM kernels)
            ops.k_linear_wgrad_group(items)
            for it, (fw, fb) in zip(items, first):
                assert torch.equal(it[2], fw)
                assert fb is None or torch.equal(it[3], fb)


CONVS = [  # (N, Cin, H, Cout, k, stride, pad, dil)
    (2, 64, 16, 64, 1, 1, 0, 1),
    (2, 64, 15, 128, 1, 2, 0, 1),
    (2, 64, 16, 64, 3, 1, 1, 1),
    (2, 32, 17, 64, 3, 2, 1, 1),
    (2, 64, 14, 64, 3, 1, 2, 2),
    (2, 3, 32, 64, 7, 2, 3, 1),
]


def _pack(w, cdtype):
    co, ci, k, _ = w.shape
    cp = max(8, (ci + 7) // 8 * 8)
    wp = torch.empty(co, k, k, cp, dtype=cdtype, device=DEV)
    wt = torch.empty(cp, k, k, co, dtype=cdtype, device=DEV)
    bias = torch.empty(co, device=DEV)
    scale = torch.empty(co, device=DEV)
    bw = torch.rand(co, device=DEV) + 0.5
    bb = torch.randn(co, device=DEV) * 0.1
    rm = torch.randn(co, device=DEV) * 0.1
    rv = torch.rand(co, device=DEV) + 0.5
    call("retr_conv_pack", ops.dcode(cdtype), ptr(w), ptr(bw), ptr(bb), ptr(rm), ptr(rv), None,
         co, ci, k, k, cp, ptr(wp), ptr(wt), ptr(bias), ptr(scale), ops._st())
    return wp, wt, bias, scale, cp, (bw, bb, rm, rv)


# Shapes large enough for the LDS-DMA tiles of gemm2.hpp (256x128, 256x64, 128x128 blocks,
# split-K weight gradients, stride-2 phase dgrad, dilation, ragged M).
BIG_CONVS = [
    (16, 64, 63, 256, 3, 1, 1, 1),
    (16, 64, 64, 64, 3, 1, 1, 1),
    (4, 128, 60, 256, 1, 1, 0, 1),
    (8, 128, 81, 128, 3, 2, 1, 1),
    (8, 256, 30, 256, 3, 1, 2, 2),
    (16, 256, 41, 512, 1, 2, 0, 1),
    # 64x64-tile rule (conv.hip prefer_tile64): layer-4 sized maps, stride-2 phases, 1x1 to / from
    # 1024 channels
    (16, 512, 20, 512, 3, 1, 1, 1),
    (16, 512, 40, 512, 3, 2, 1, 1),
    (8, 1024, 40, 256, 1, 1, 0, 1),
    (8, 256, 40, 1024, 1, 1, 0, 1),
    (16, 512, 20, 2048, 1, 1, 0, 1),
]


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 5e-6), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("cfg", CONVS)
def test_conv_fwd_dgrad_wgrad(dtype, tol, cfg):
    _check_conv(dtype, tol, cfg)


@pytest.mark.parametrize("cfg", BIG_CONVS)
def test_conv_big_bf16(cfg):
    _check_conv(torch.bfloat16, 2e-2, cfg)


def _check_conv(dtype, tol, cfg):
    N, Ci, H, Co, k, s, p, d = cfg
    g = torch.Generator(device="cpu").manual_seed(sum(cfg))
    x = torch.randn(N, Ci, H, H, generator=g)
    w = torch.randn(Co, Ci, k, k, generator=g) / math.sqrt(Ci * k * k)
    wd = w.to(DEV)
    wp, wt, bias, scale, cp, (bw, bb, rm, rv) = _pack(wd, dtype)
    # reference (CPU fp32) with the folded weights as the kernel sees them
    weff = (wp.float()[..., :Ci].permute(0, 3, 1, 2)).cpu()
    xr = x.to(dtype).float()
    ref = F.conv2d(xr, weff, stride=s, padding=p, dilation=d) + bias.cpu().view(1, -1, 1, 1)
    ref = torch.relu(ref)
    xn = torch.zeros(N, H, H, cp, dtype=dtype, device=DEV)
    xn[..., :Ci] = x.permute(0, 2, 3, 1).to(DEV).to(dtype)
    OH = (H + 2 * p - d * (k - 1) - 1) // s + 1
    y = torch.empty(N, OH, OH, Co, dtype=dtype, device=DEV)
    call("retr_conv2d_fwd", ops.dcode(dtype), ptr(xn), N, H, H, cp, ptr(wp), ptr(bias), None,
         ptr(y), Co, k, k, s, p, d, 1, ops._st())
    assert rel_err(y.permute(0, 3, 1, 2), ref) < tol
    # backward: dgrad and wgrad of the folded conv
    gy = torch.randn(N, Co, OH, OH, generator=g)
    gyc = gy.to(dtype).float()
    xreq = xr.clone().requires_grad_(True)
    wreq = weff.clone().requires_grad_(True)
    F.conv2d(xreq, wreq, stride=s, padding=p, dilation=d).backward(gyc)
    gn = gy.permute(0, 2, 3, 1).contiguous().to(DEV).to(dtype)
    if Ci % 8 == 0:
        dx = torch.empty(N, H, H, cp, dtype=dtype, device=DEV)
        call("retr_conv2d_dgrad", ops.dcode(dtype), ptr(gn), N, H, H, cp, ptr(wt), ptr(dx), Co,
             k, k, s, p, d, None, None, ops._st())
        assert rel_err(dx.permute(0, 3, 1, 2), xreq.grad) < tol
    splits = _lib.load().retr_conv2d_wgrad_splits(ops.dcode(dtype), N, H, H, cp, Co, k, k, s,
                                                  p, d)
    assert splits >= 1
    ws = torch.full((splits, Co, k * k * cp), float("nan"), device=DEV)   # overwritten
    call("retr_conv2d_wgrad", ops.dcode(dtype), ptr(gn), ptr(xn), N, H, H, cp, ptr(ws), Co, k, k,
         s, p, d, ops._st())
    grad = torch.empty(Co, Ci, k, k, device=DEV)
    call("retr_conv_wgrad_unpack", ptr(ws), None, ptr(grad), Co, Ci, cp, k, k, 0, splits,
         ops._st())
    assert rel_err(grad, wreq.grad) < tol


@pytest.mark.parametrize("cfg", CONVS[2:] + BIG_CONVS[:2] + BIG_CONVS[3:5] + BIG_CONVS[6:8])
def test_conv_wgrad_b32_loader_bitwise(cfg):
    """The 32-bit-offset weight-gradient loader (ConvWgradB32) visits the same pixels in the same
    K order as the 64-bit one: identical split-K slabs (RETR_TUNE_WGRAD_B32 = 1 selects the
    64-bit loader)."""
    N, Ci, H, Co, k, s, p, d = cfg
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(sum(cfg) + 7)
    cp = max(8, (Ci + 7) // 8 * 8)
    OH = (H + 2 * p - d * (k - 1) - 1) // s + 1
    xn = torch.zeros(N, H, H, cp, dtype=bf, device=DEV)
    xn[..., :Ci] = torch.randn(N, H, H, Ci, generator=g).to(DEV).to(bf)
    gn = torch.randn(N, OH, OH, Co, generator=g).to(DEV).to(bf)
    lib = _lib.load()
    splits = lib.retr_conv2d_wgrad_splits(ops.dcode(bf), N, H, H, cp, Co, k, k, s, p, d)
    out = []
    try:
        for knob in (0, 1):
            lib.retr_tune(16, knob)
            ws = torch.full((splits, Co, k * k * cp), float("nan"), device=DEV)
            call("retr_conv2d_wgrad", ops.dcode(bf), ptr(gn), ptr(xn), N, H, H, cp, ptr(ws), Co,
                 k, k, s, p, d, ops._st())
            out.append(ws)
    finally:
        lib.retr_tune(16, 0)
    assert not torch.isnan(out[0]).any()
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("M,C", [(37, 64), (512, 256), (130, 512), (6400, 256), (4100, 512)])
def test_layernorm(dtype, tol, M, C):
    g = torch.Generator(device="cpu").manual_seed(M * C)
    x = (torch.randn(M, C, generator=g) * 3 + 1).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    pos = torch.randn(16, C, generator=g).to(DEV)
    norm = torch.nn.LayerNorm(C).to(DEV)
    norm.weight.data.copy_(gamma)
    norm.bias.data.copy_(beta)
    xr = x.clone().requires_grad_(True)
    posr = pos.clone().requires_grad_(True)
    n, npos = ops.ln_pos(xr, norm, dtype, pos=posr, period=16)
    xt = x.clone().requires_grad_(True)
    pt = pos.clone().requires_grad_(True)
    nt = F.layer_norm(xt, (C,), gamma, beta, 1e-5)
    rows = torch.arange(M, device=DEV) % 16
    npt = nt + pt[rows]
    assert rel_err(n, nt) < tol and rel_err(npos, npt) < tol
    g1 = torch.randn(M, C, generator=g).to(DEV)
    g2 = torch.randn(M, C, generator=g).to(DEV)
    (n.float() * g1 + npos.float() * g2).sum().backward()
    (nt * g1 + npt * g2).sum().backward()
    assert rel_err(xr.grad, xt.grad) < 5 * tol
    assert rel_err(posr.grad, pt.grad) < 5 * tol
    gt = gamma.clone().requires_grad_(True)
    bt = beta.clone().requires_grad_(True)
    nt2 = F.layer_norm(x, (C,), gt, bt, 1e-5)
    (nt2 * g1 + (nt2 + pos[rows]) * g2).sum().backward()
    assert rel_err(norm.weight.grad, gt.grad) < 5 * tol
    assert rel_err(norm.bias.grad, bt.grad) < 5 * tol


@pytest.mark.parametrize("M,C,F,prev", [(6400, 256, 2048, True), (2048, 256, 2048, False),
                                        (600, 512, 2048, True)])
def test_layernorm_bwd_from_dgrad_slabs_bitwise(M, C, F, prev):
    """The FFN block's pre-norm LayerNorm backward fed by the up-projection's split-K data
    gradient slabs (retr_linear_dgrad_slabs + retr_layernorm_bwd_slabs) against the split-K
    data gradient with its bf16 slab epilogue + retr_layernorm_bwd2: dx, the previous block's
    dropout(dx) and the dgamma / dbeta partial rows bitwise equal."""
    import ctypes
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(M + C)
    dh = torch.randn(M, F, generator=g).to(DEV, bf)
    w1 = (torch.randn(F, C, generator=g) / math.sqrt(F)).to(DEV, bf)     # W1 [F][C]
    x = (torch.randn(M, C, generator=g) * 2 + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    addend = torch.randn(M, C, generator=g).to(DEV)
    lib = _lib.load()
    sp = int(lib.retr_linear_splits(1, M, C, F))
    assert sp > 1
    nws = int(lib.retr_layernorm_bwd_workspace(M, C))
    outs = []
    for slab in (False, True):
        dx = torch.full((M, C), float("nan"), device=DEV)
        dxd = torch.full((M, C), float("nan"), device=DEV, dtype=bf) if prev else None
        ws = torch.zeros(nws // 4 + 64, device=DEV)
        sws = torch.empty(sp, M, C, device=DEV)
        nparts = ctypes.c_int(0)
        pdrop = (0.1, 4321) if prev else (0.0, 0)
        if slab:
            call("retr_linear_dgrad_slabs", 1, ptr(dh), F, ptr(w1), C, M, F, C, 0, ptr(sws), sp,
                 ops._st())
            call("retr_layernorm_bwd_slabs", ptr(sws), sp, ptr(x), C, ptr(gamma), ptr(mean),
                 ptr(rstd), M, C, ptr(dx), C, ptr(addend), None, None, ptr(ws), ptr(dxd), C,
                 pdrop[0], pdrop[1], ctypes.addressof(nparts), ops._st())
        else:
            dn = torch.empty(M, C, device=DEV, dtype=bf)
            call("retr_linear_dgrad_splitk", 1, ptr(dh), F, ptr(w1), C, ptr(dn), C, 0, M, F, C,
                 None, 0, 0, None, 0, 0, ptr(sws), sp, ops._st())
            call("retr_layernorm_bwd2", 1, ptr(dn), None, C, ptr(x), C, ptr(gamma), ptr(mean),
                 ptr(rstd), M, C, ptr(dx), C, ptr(addend), None, None, ptr(ws), ptr(dxd), C,
                 pdrop[0], pdrop[1], ctypes.addressof(nparts), ops._st())
        torch.cuda.synchronize()
        n = nparts.value
        outs.append((dx, dxd, ws[: 2 * C * n].clone(), n))
    (a, ad, ap, an), (b, bd, bp, bn) = outs
    assert an == bn and an > 0
    assert not torch.isnan(a).any() and torch.equal(a, b)
    if prev:
        assert torch.equal(ad, bd)
    assert torch.equal(ap, bp)


def _attn_ref(q, k, v, H, kpm, causal):
    B, Lq, C = q.shape
    Lk = k.shape[1]
    hd = C // H
    qh = q.view(B, Lq, H, hd).transpose(1, 2) * (1.0 / math.sqrt(hd))
    kh = k.view(B, Lk, H, hd).transpose(1, 2)
    vh = v.view(B, Lk, H, hd).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2)
    if kpm is not None:
        s = s.masked_fill(kpm.bool()[:, None, None, :], float("-inf"))
    if causal:
        cm = torch.ones(Lq, Lk, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(cm, float("-inf"))
    p = s.softmax(-1)
    return (p @ vh).transpose(1, 2).reshape(B, Lq, C), p.mean(1)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("B,H,Lq,Lk,hd,causal,masked", [
    (2, 8, 16, 4, 8, False, True), (2, 8, 128, 128, 16, True, True),
    (3, 8, 100, 77, 32, False, True), (2, 8, 128, 400, 32, False, False),
    (2, 4, 70, 70, 64, False, True)])
def test_attention(dtype, tol, B, H, Lq, Lk, hd, causal, masked):
    g = torch.Generator(device="cpu").manual_seed(B * Lq + Lk + hd)
    C = H * hd
    q = torch.randn(B, Lq, C, generator=g).to(DEV).to(dtype)
    k = torch.randn(B, Lk, C, generator=g).to(DEV).to(dtype)
    v = torch.randn(B, Lk, C, generator=g).to(DEV).to(dtype)
    kpm = None
    if masked:
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[:, Lk - Lk // 4:] = 1
        kpm = kpm.to(DEV)
    o = torch.empty(B * Lq, C, dtype=dtype, device=DEV)
    lse = torch.empty(B * H * Lq, device=DEV)
    probs = torch.empty(B, Lq, Lk, device=DEV)
    ops.k_attention_fwd(q.view(-1, C), k.view(-1, C), v.view(-1, C), o, B, H, Lq, Lk, hd, kpm,
                        causal, 0.0, 0, lse, probs)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    ref, pref = _attn_ref(qr, kr, vr, H, kpm, causal)
    assert rel_err(o.view(B, Lq, C), ref) < tol
    assert rel_err(probs, pref) < tol
    do = torch.randn(B, Lq, C, generator=g).to(DEV).to(dtype)
    ref.backward(do.float())
    dq = torch.empty_like(o)
    dk = torch.empty(B * Lk, C, dtype=dtype, device=DEV)
    dv = torch.empty_like(dk)
    ops.k_attention_bwd(q.view(-1, C), k.view(-1, C), v.view(-1, C), o, do.view(-1, C), lse, dq,
                        dk, dv, B, H, Lq, Lk, hd, kpm, causal, 0.0, 0)
    assert rel_err(dq.view(B, Lq, C), qr.grad) < 3 * tol
    assert rel_err(dk.view(B, Lk, C), kr.grad) < 3 * tol
    assert rel_err(dv.view(B, Lk, C), vr.grad) < 3 * tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("B,H,Lk,Lmax,hd,masked", [
    (2, 8, 1, 128, 32, False), (3, 8, 77, 128, 32, False), (2, 8, 400, 400, 32, True),
    (4, 4, 128, 128, 64, True), (2, 8, 19, 20, 8, False)])
def test_attention_decode(dtype, tol, B, H, Lk, Lmax, hd, masked):
    """Single-query attention over a [B][Lmax] key cache (first Lk rows valid)."""
    g = torch.Generator(device="cpu").manual_seed(B * Lk + hd)
    C = H * hd
    q = torch.randn(B, 1, C, generator=g).to(DEV).to(dtype)
    kc = torch.randn(B, Lmax, C, generator=g).to(DEV).to(dtype)
    vc = torch.randn(B, Lmax, C, generator=g).to(DEV).to(dtype)
    kpm = None
    if masked:
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[:, Lk - Lk // 4:] = 1
        kpm = kpm.to(DEV)
    o = torch.empty(B, C, dtype=dtype, device=DEV)
    call("retr_attention_decode", ops.dcode(dtype), ptr(q), C, ptr(kc), C, ptr(vc), C, ptr(o), C,
         B, H, Lk, Lmax, hd, ptr(kpm), 1, None, ops._st())
    ref, _ = _attn_ref(q.float(), kc[:, :Lk].float(), vc[:, :Lk].float(), H, kpm, False)
    assert rel_err(o.view(B, 1, C), ref) < tol


def test_attention_dropout_statistics():
    B, H, L, hd = 2, 8, 128, 32
    C = H * hd
    q = torch.zeros(B * L, C, device=DEV)
    k = torch.zeros(B * L, C, device=DEV)
    v = torch.ones(B * L, C, device=DEV)
    o = torch.empty(B * L, C, device=DEV)
    lse = torch.empty(B * H * L, device=DEV)
    ops.k_attention_fwd(q, k, v, o, B, H, L, L, hd, None, False, 0.1, 1234, lse)
    # each output = mean over keys of keep/(1-p): expectation 1, row-wise mean ~1
    assert abs(o.mean().item() - 1.0) < 0.02
    o2 = torch.empty_like(o)
    ops.k_attention_fwd(q, k, v, o2, B, H, L, L, hd, None, False, 0.1, 1234, lse)
    assert torch.equal(o, o2)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
def test_cross_entropy_and_argmax(dtype, tol):
    B, T, V = 3, 16, 30522
    g = torch.Generator(device="cpu").manual_seed(7)
    Vp = (V + 63) // 64 * 64
    buf = torch.zeros(B * T, Vp, device=DEV, dtype=dtype)
    buf[:, :V] = (torch.randn(B * T, V, generator=g) * 2).to(DEV).to(dtype)
    logits = buf[:, :V].view(B, T, V).requires_grad_(False)
    tgt = torch.randint(0, V, (B, T), generator=g).to(DEV)
    x = logits.clone().float().requires_grad_(True)
    lref = F.cross_entropy(x.permute(0, 2, 1), tgt)
    lref.backward()
    lt = logits.detach().requires_grad_(True)
    loss = ops.cross_entropy(lt.permute(0, 2, 1), tgt)
    assert abs(loss.item() - lref.item()) < tol * abs(lref.item())
    loss.backward()
    assert rel_err(lt.grad.float(), x.grad) < 5 * tol
    am = ops.argmax_rows(buf[:, :V])
    assert torch.equal(am, buf[:, :V].float().argmax(-1))


def _mix32(x):
    x = x.astype(np.uint64) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def _mix24(x):
    """common.hpp mix24: the finaliser on 24-bit multiplies (v_mul_u32_u24)."""
    x = x.astype(np.uint64) & 0xFFFFFFFF
    x ^= x >> 16
    x = ((x & 0xFFFFFF) * 0xEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = ((x & 0xFFFFFF) * 0x6CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def attn_keep_mask(seed, B, H, Lq, Lk, p):
    """numpy restatement of the fused attention kernels' dropout keep mask (csrc/common.hpp
    attn_row_key / attn_pair_bits / attn_keep): [B, H, Lq, Lk] bool."""
    thresh = int(np.float32(min(np.float32(p) * np.float32(4294967296.0), 4294967295.0)))
    th16 = (thresh + 0x8000) >> 16
    rows = np.arange(B * H * Lq, dtype=np.uint64)
    s_lo, s_hi = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    rk = _mix32(s_lo ^ _mix32((rows * 0x9E3779B9 + s_hi) & 0xFFFFFFFF))
    keys = np.arange(Lk, dtype=np.uint64)
    bits = _mix24((rk[:, None] + ((keys[None, :] >> 1) & 0xFFFFFF) * 0xEBCA77) & 0xFFFFFFFF)
    half = np.where(keys[None, :] & 1, bits >> 16, bits & 0xFFFF)
    return torch.from_numpy((half >= th16).reshape(B, H, Lq, Lk))


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("B,H,Lq,Lk,hd,causal,masked", [
    (2, 8, 400, 400, 32, False, True), (2, 8, 128, 128, 32, True, True),
    (2, 8, 128, 196, 64, False, True), (1, 8, 130, 625, 64, False, True)])
def test_attention_dropout_exact_mask(dtype, tol, B, H, Lq, Lk, hd, causal, masked):
    """Forward and backward with dropout p=0.1 against torch on the kernels' own keep mask
    (restated in numpy): the backward regenerates exactly the forward's mask."""
    from retr_amd import ops
    g = torch.Generator(device="cpu").manual_seed(7 * Lq + Lk + hd)
    C = H * hd
    q = torch.randn(B, Lq, C, generator=g).to(DEV).to(dtype)
    k = torch.randn(B, Lk, C, generator=g).to(DEV).to(dtype)
    v = torch.randn(B, Lk, C, generator=g).to(DEV).to(dtype)
    kpm = None
    if masked:
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[:, Lk - Lk // 5:] = 1
        kpm = kpm.to(DEV)
    seed, p = 0x1234567887654321, 0.1
    base = int(ops.seed_base().item())                 # dropout seed = op seed + step seed
    keep = attn_keep_mask((seed + base) & (2 ** 64 - 1), B, H, Lq, Lk, p).to(DEV)
    o = torch.empty(B * Lq, C, dtype=dtype, device=DEV)
    lse = torch.empty(B * H * Lq, device=DEV)
    ops.k_attention_fwd(q.view(-1, C), k.view(-1, C), v.view(-1, C), o, B, H, Lq, Lk, hd, kpm,
                        causal, p, seed, lse)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    qh = qr.view(B, Lq, H, hd).transpose(1, 2) * (1.0 / math.sqrt(hd))
    kh = kr.view(B, Lk, H, hd).transpose(1, 2)
    vh = vr.view(B, Lk, H, hd).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2)
    if kpm is not None:
        s = s.masked_fill(kpm.bool()[:, None, None, :], float("-inf"))
    if causal:
        s = s.masked_fill(torch.ones(Lq, Lk, dtype=torch.bool, device=DEV).triu(1),
                          float("-inf"))
    pm = s.softmax(-1) * keep / (1 - p)
    ref = (pm @ vh).transpose(1, 2).reshape(B, Lq, C)
    assert rel_err(o.view(B, Lq, C), ref) < tol
    do = torch.randn(B, Lq, C, generator=g).to(DEV).to(dtype)
    ref.backward(do.float())
    dq = torch.empty_like(o)
    dk = torch.empty(B * Lk, C, dtype=dtype, device=DEV)
    dv = torch.empty_like(dk)
    ops.k_attention_bwd(q.view(-1, C), k.view(-1, C), v.view(-1, C), o, do.view(-1, C), lse, dq,
                        dk, dv, B, H, Lq, Lk, hd, kpm, causal, p, seed)
    assert rel_err(dq.view(B, Lq, C), qr.grad) < 3 * tol
    assert rel_err(dk.view(B, Lk, C), kr.grad) < 3 * tol
    assert rel_err(dv.view(B, Lk, C), vr.grad) < 3 * tol


def test_attention_fully_masked_rows_nan():
    """A query row whose keys are all padded is NaN (torch softmax of an all -inf row)."""
    from retr_amd import ops
    B, H, L, hd = 2, 8, 64, 32
    C = H * hd
    q = torch.randn(B * L, C, device=DEV).to(torch.bfloat16)
    kpm = torch.zeros(B, L, dtype=torch.uint8, device=DEV)
    kpm[1] = 1
    o = torch.empty(B * L, C, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * L, device=DEV)
    ops.k_attention_fwd(q, q, q, o, B, H, L, L, hd, kpm, False, 0.0, 0, lse)
    assert torch.isfinite(o[:L].float()).all() and torch.isnan(o[L:].float()).all()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("view", [True, False])
def test_linear_dgrad_split_reduction(dtype, tol, view):
    """dx = gate(dy W) with the vocabulary-long reduction split into ordered fp32 slabs (the MLP
    head's data gradient), W given row-major (read transposed) or as a materialised W^T."""
    M, N, K = 300, 30528, 512
    g = torch.Generator(device="cpu").manual_seed(9)
    dy = torch.randn(M, N, generator=g).to(DEV).to(dtype)
    w = (torch.randn(N, K, generator=g) / 100).to(DEV).to(dtype)
    gate = torch.randn(M, K, generator=g).to(DEV).to(dtype)
    dx = torch.empty(M, K, dtype=dtype, device=DEV)
    wt = ops._TView(w) if view else w.t().contiguous()
    ops.k_linear_dgrad(dy, wt, dx, gate=gate)
    ref = (dy.float() @ w.float()) * (gate.float() > 0)
    assert rel_err(dx.float(), ref) < tol
    dx2 = torch.empty_like(dx)
    ops.k_linear_dgrad(dy, wt, dx2, gate=gate)
    assert torch.equal(dx, dx2)                      # slabs added in order: deterministic


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stem_layout_and_maxpool(dtype):
    """NCHW fp32 image -> NHWC (channels zero-padded to 8) and MaxPool2d(3, 2, 1) on NHWC
    (torchvision's stem, models/backbone.py:65-69) against torch."""
    g = torch.Generator(device="cpu").manual_seed(4)
    N, C, H, W = 3, 3, 37, 42
    x = torch.randn(N, C, H, W, generator=g).to(DEV)
    y = torch.empty(N, H, W, 8, dtype=dtype, device=DEV)
    call("retr_nchw_to_nhwc", ops.dcode(dtype), ptr(x), ptr(y), N, C, H, W, 8, ops._st())
    ref = torch.zeros(N, H, W, 8, device=DEV)
    ref[..., :C] = x.permute(0, 2, 3, 1)
    assert torch.equal(y.float(), ref.to(dtype).float())
    Cm, Hm, Wm = 64, 33, 40
    xm = torch.randn(N, Hm, Wm, Cm, generator=g).to(DEV).to(dtype)
    OH, OW = (Hm - 1) // 2 + 1, (Wm - 1) // 2 + 1
    ym = torch.empty(N, OH, OW, Cm, dtype=dtype, device=DEV)
    call("retr_maxpool3x3s2", ops.dcode(dtype), ptr(xm), ptr(ym), N, Hm, Wm, Cm, OH, OW, ops._st())
    refm = F.max_pool2d(xm.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(ym.float(), refm)


@pytest.mark.parametrize("B,H,Lq,Lk,hd,causal,masked,p", [
    (16, 8, 400, 400, 32, False, True, 0.1), (16, 8, 128, 400, 32, False, True, 0.1),
    (16, 8, 128, 128, 32, True, False, 0.1), (3, 8, 100, 77, 32, False, True, 0.0),
    (2, 8, 130, 200, 64, False, True, 0.1), (2, 8, 200, 200, 64, True, True, 0.0)])
def test_attention_resident_equals_streaming(B, H, Lq, Lk, hd, causal, masked, p):
    """The LDS-resident bf16 kernels (attention2.hip fwd3/dq3/dkdv3, unsplit) compute the
    streaming kernels' fragments in the same order: outputs, lse and all three gradients
    bit-identical; the default split backward agrees to bf16 rounding."""
    g = torch.Generator(device="cpu").manual_seed(Lq * 7 + Lk)
    C = H * hd
    bf = torch.bfloat16
    q, k, v, do = (torch.randn(B * L, C, generator=g).to(DEV).to(bf) for L in (Lq, Lk, Lk, Lq))
    kpm = None
    if masked:
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[:, Lk - Lk // 5:] = 1
        kpm = kpm.to(DEV)
    outs = []
    for mode, split in ((1, 1), (2, 1), (0, 0)):
        _lib.load().retr_tune(5, mode)
        _lib.load().retr_tune(10, split)
        try:
            o = torch.empty(B * Lq, C, dtype=bf, device=DEV)
            lse = torch.empty(B * H * Lq, device=DEV)
            ops.k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, causal, p, 1234, lse)
            dq, dk, dv = (torch.empty_like(t) for t in (q, k, v))
            ops.k_attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, hd, kpm, causal, p,
                                1234)
            torch.cuda.synchronize()
            outs.append((o, lse, dq, dk, dv))
        finally:
            _lib.load().retr_tune(5, 0)
            _lib.load().retr_tune(2, 0)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    # the default split backward (two waves per 32 rows, even + odd tile partials added at the
    # end): the same products summed in another fixed order
    for a, b in zip(outs[2], outs[1]):
        e = ((a.float() - b.float()).norm() / (b.float().norm() + 1e-30)).item()
        assert e < 5e-3, e


@pytest.mark.parametrize("H,Ci,Co,k,p", [(16, 64, 128, 1, 0), (15, 64, 128, 1, 0),
                                          (16, 32, 64, 3, 1)])
def test_conv_dgrad_stride2_addend_gate(H, Ci, Co, k, p):
    """Stride-2 data gradient with the residual addend and the ReLU gate (the downsample branch
    of a bottleneck): tap-less phases of a 1x1 kernel are filled elementwise."""
    N, s = 2, 2
    g = torch.Generator(device="cpu").manual_seed(H + Ci + k)
    bf = torch.bfloat16
    w = torch.randn(Co, Ci, k, k, generator=g) / math.sqrt(Ci * k * k)
    wp, wt, bias, scale, cp, _ = _pack(w.to(DEV), bf)
    weff = (wp.float()[..., :Ci].permute(0, 3, 1, 2)).cpu()
    OH = (H + 2 * p - (k - 1) - 1) // s + 1
    gy = torch.randn(N, Co, OH, OH, generator=g).to(bf).float()
    add = torch.randn(N, H, H, Ci, generator=g).to(bf)
    gate = torch.randn(N, H, H, Ci, generator=g).to(bf)
    xreq = torch.zeros(N, Ci, H, H, requires_grad=True)
    F.conv2d(xreq, weff, stride=s, padding=p).backward(gy)
    ref = (xreq.grad.permute(0, 2, 3, 1) + add.float()) * (gate.float() > 0)
    gn = gy.permute(0, 2, 3, 1).contiguous().to(DEV).to(bf)
    dx = torch.full((N, H, H, cp), float("nan"), dtype=bf, device=DEV)
    add_d, gate_d = add.to(DEV), gate.to(DEV)     # kept alive across the launch
    call("retr_conv2d_dgrad", ops.dcode(bf), ptr(gn), N, H, H, cp, ptr(wt), ptr(dx), Co, k, k, s,
         p, 1, ptr(add_d), ptr(gate_d), ops._st())
    assert rel_err(dx.float().cpu(), ref) < 1e-2
    # in place (resnet.py's first blocks): dx already holds gate(addend) everywhere and the
    # stride-2 data gradient is added at the pixels its taps reach -- bitwise the out-of-place
    # result (gate(a + b) = gate(a) + b where the gate is 1, 0 elsewhere)
    dx2 = (add_d.float() * (gate_d.float() > 0)).to(bf)
    call("retr_conv2d_dgrad", ops.dcode(bf), ptr(gn), N, H, H, cp, ptr(wt), ptr(dx2), Co, k, k, s,
         p, 1, ptr(dx2), ptr(gate_d), ops._st())
    torch.cuda.synchronize()
    assert torch.equal(dx2, dx)


@pytest.mark.parametrize("M,N,K", [(6400, 256, 2048), (2048, 256, 2048), (1000, 200, 1536)])
def test_linear_splitk_fwd_dgrad(M, N, K):
    """Split-K forward (bias + dropout + residual on the ordered slab sum) and data gradient
    (addend + gate): against fp32 torch, against the single-pass kernels with the same dropout
    mask, and bit-identical on a repeat."""
    bf = torch.bfloat16
    assert _lib.load().retr_linear_splits(1, M, N, K) > 1
    g = torch.Generator(device="cpu").manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(DEV).to(bf)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV).to(bf)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    y = torch.empty(M, N, device=DEV)
    ops.k_linear_fwd(x, w, b, y, res=res)
    assert rel_err(y, x.float() @ w.float().t() + b + res) < 1e-2
    y1, y2 = torch.empty_like(y), torch.empty_like(y)
    ops.k_linear_fwd(x, w, b, y1, res=res, drop_p=0.1, seed=77)
    ops.k_linear_fwd(x, w, b, y2, res=res, drop_p=0.1, seed=77)
    assert torch.equal(y1, y2)
    ys = torch.empty_like(y)
    call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(ys), N, 1, M, N, K, 0, ptr(res),
         N, 0.1, 77, ops._st())
    assert rel_err(y1, ys) < 1e-2                  # same dropout mask as the single pass
    # data gradient: dx[M][K] = gate(dy[M][N] W[N][K] + addend): reduction N... use W^T shapes
    dy = torch.randn(M, K, generator=g).to(DEV).to(bf)        # [M][K] -> dx [M][N] over K
    add = torch.randn(M, N, generator=g).to(DEV).to(bf)
    gate = torch.randn(M, N, generator=g).to(DEV).to(bf)
    dx = torch.empty(M, N, dtype=bf, device=DEV)
    ops.k_linear_dgrad(dy, ops._TView(w.t().contiguous()), dx, addend=add, gate=gate)
    ref = (dy.float() @ w.float().t() + add.float()) * (gate.float() > 0)
    assert rel_err(dx.float(), ref) < 1e-2
    dx2 = torch.empty_like(dx)
    ops.k_linear_dgrad(dy, ops._TView(w.t().contiguous()), dx2, addend=add, gate=gate)
    assert torch.equal(dx, dx2)


def test_linear_dropout_mask_regenerated_by_backward():
    """The residual-branch dropout of a linear forward (GEMM epilogue) and the backward's
    retr_dropout_apply draw the same keep mask from (seed, row, column); keep rate ~ 1 - p."""
    M, N, K, p, seed = 3000, 256, 64, 0.1, 12345
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(M, K, generator=g).to(DEV).to(torch.bfloat16)
    w = torch.randn(N, K, generator=g).to(DEV).to(torch.bfloat16)
    b = torch.full((N,), 10.0, device=DEV)                 # branch never exactly zero
    res = torch.zeros(M, N, device=DEV)
    y = torch.empty(M, N, device=DEV)
    ops.k_linear_fwd(x, w, b, y, res=res, drop_p=p, seed=seed)
    kept_fwd = y != 0
    ones = torch.ones(M, N, device=DEV)
    m = torch.empty(M, N, device=DEV)
    ops.k_dropout_apply(ones, m, p, seed)
    kept_bwd = m != 0
    assert torch.equal(kept_fwd, kept_bwd)
    assert abs(kept_bwd.float().mean().item() - (1 - p)) < 5e-3
    assert torch.allclose(m[kept_bwd], torch.full_like(m[kept_bwd], 1 / (1 - p)))


def test_argmax_split_matches_single_pass():
    """Split (16 segments per row) first-index argmax == the one-block-per-row kernel ==
    torch.argmax on bf16 decode logits, incl. ties across segments and a NaN row."""
    M, V, Vp = 64, 30522, 30528
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.randn(M, Vp, generator=g).to(torch.bfloat16)
    x[:, V:] = 0
    x[3, 100] = x[3, 25000] = 50.0                  # tie: first index wins
    x[5, 29999] = float("nan")                      # NaN wins (torch semantics)
    x = x.to(DEV)
    ws = torch.empty(_lib.load().retr_argmax_workspace(M) // 4, device=DEV)
    a = torch.empty(M, dtype=torch.long, device=DEV)
    b = torch.empty(M, dtype=torch.long, device=DEV)
    call("retr_argmax_rows_ws", 1, ptr(x), Vp, M, V, ptr(a), ptr(ws), ops._st())
    call("retr_argmax_rows", 1, ptr(x), Vp, M, V, ptr(b), ops._st())
    assert torch.equal(a, b)
    assert torch.equal(a.cpu(), x[:, :V].float().cpu().argmax(1))
    assert int(a[3]) == 100 and int(a[5]) == 29999


@pytest.mark.parametrize("dt", [1, 0])
def test_conv_pack_group_matches_single(dt):
    """Grouped weight packing (one launch for many convs; the tiled kernel's 16-byte loads and
    stores) == per-conv retr_conv_pack, bf16 and fp32 images."""
    odt = torch.bfloat16 if dt == 1 else torch.float32
    shapes = [(64, 3, 7, 8), (128, 64, 3, 64), (256, 128, 1, 128), (512, 512, 3, 512)]
    arr = (_lib.ConvPackDesc * len(shapes))()
    outs, refs, keep = [], [], []
    for i, (co, ci, k, cp) in enumerate(shapes):
        w = torch.randn(co, ci, k, k, device=DEV)
        bw, bb = torch.rand(co, device=DEV) + 0.5, torch.randn(co, device=DEV)
        rm, rv = torch.randn(co, device=DEV), torch.rand(co, device=DEV) + 0.5
        keep += [w, bw, bb, rm, rv]
        o = [torch.empty(co, k, k, cp, dtype=odt, device=DEV),
             torch.empty(cp, k, k, co, dtype=odt, device=DEV),
             torch.empty(co, device=DEV), torch.empty(co, device=DEV)]
        r = [torch.empty_like(t) for t in o]
        call("retr_conv_pack", dt, ptr(w), ptr(bw), ptr(bb), ptr(rm), ptr(rv), None, co, ci, k, k,
             cp, ptr(r[0]), ptr(r[1]), ptr(r[2]), ptr(r[3]), ops._st())
        d = arr[i]
        d.w, d.bn_w, d.bn_b, d.bn_rm, d.bn_rv = ptr(w), ptr(bw), ptr(bb), ptr(rm), ptr(rv)
        d.w_out, d.wt_out, d.bias_out, d.scale_out = (ptr(t) for t in o)
        d.Co, d.Ci, d.KH, d.KW, d.Cp = co, ci, k, k, cp
        outs.append(o)
        refs.append(r)
    call("retr_conv_pack_group", dt, len(shapes), arr, ops._st())
    for o, r in zip(outs, refs):
        for a, b in zip(o, r):
            assert torch.equal(a, b)


@pytest.mark.parametrize("N,H,W", [(2, 64, 64), (3, 38, 50), (16, 224, 224)])
def test_stem_space_to_depth(N, H, W):
    """bf16 stem as a 4x4 stride-1 conv over the space-to-depth image (retr_nchw_to_s2d16 +
    retr_stem_s2d_weights + retr_conv2d_fwd_out) == the 7x7 stride-2 conv over NHWC8: same bf16
    operands and products (only the fp32 summation order differs), and both against fp32 torch."""
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(N * H + W)
    img = torch.randn(N, 3, H, W, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) / math.sqrt(147)
    wp, _, bias, _, cp, _ = _pack(w.to(DEV), bf)
    imd = img.to(DEV)
    OH, OW = H // 2, W // 2
    x8 = torch.empty(N, H, W, 8, dtype=bf, device=DEV)
    call("retr_nchw_to_nhwc", ops.dcode(bf), ptr(imd), ptr(x8), N, 3, H, W, 8, ops._st())
    y_ref = torch.empty(N, OH, OW, 64, dtype=bf, device=DEV)
    call("retr_conv2d_fwd", ops.dcode(bf), ptr(x8), N, H, W, 8, ptr(wp), ptr(bias), None,
         ptr(y_ref), 64, 7, 7, 2, 3, 1, 1, ops._st())
    xs = torch.full((N, OH, OW, 16), float("nan"), dtype=bf, device=DEV)
    call("retr_nchw_to_s2d16", ptr(imd), ptr(xs), N, 3, H, W, ops._st())
    assert torch.equal(xs[..., 12:].float(), torch.zeros(N, OH, OW, 4, device=DEV))
    ref_s2d = imd.to(bf).view(N, 3, OH, 2, OW, 2).permute(0, 2, 4, 3, 5, 1).reshape(N, OH, OW, 12)
    assert torch.equal(xs[..., :12], ref_s2d)
    w2 = torch.empty(64, 4, 4, 16, dtype=bf, device=DEV)
    call("retr_stem_s2d_weights", ptr(wp), ptr(w2), 64, cp, ops._st())
    y = torch.empty(N, OH, OW, 64, dtype=bf, device=DEV)
    call("retr_conv2d_fwd_out", ops.dcode(bf), ptr(xs), N, OH, OW, 16, ptr(w2), ptr(bias), None,
         ptr(y), 64, 4, 4, 1, 2, 1, OH, OW, 1, ops._st())
    torch.cuda.synchronize()
    assert rel_err(y.float(), y_ref.float()) < 2e-3
    weff = wp.float()[..., :3].permute(0, 3, 1, 2).cpu()
    ref = torch.relu(F.conv2d(img.to(bf).float(), weff, stride=2, padding=3)
                     + bias.cpu().view(1, -1, 1, 1))
    assert rel_err(y.permute(0, 3, 1, 2).float().cpu(), ref) < 1e-2


@pytest.mark.parametrize("N,H2,W2", [(2, 320, 320), (3, 19, 25), (2, 112, 112), (1, 32, 48),
                                     (4, 17, 16)])
def test_stem_pool_fused_equals_conv_then_maxpool(N, H2, W2):
    """retr_stem_pool_fwd (space-to-depth conv + bias + ReLU + MaxPool(3, 2, 1) in one launch,
    csrc/stem.hip) == retr_conv2d_fwd_out + retr_maxpool3x3s2 bitwise, at the cfg2 size, ragged
    pooled tiles (odd sizes, partial 8x16 tiles) and the cfg5 decode size (112 = 224 / 2)."""
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + H2 * 7 + W2)
    xs = torch.randn(N, H2, W2, 16, generator=g)
    xs[..., 12:] = 0
    xs = xs.to(DEV).to(bf)
    w2 = (torch.randn(64, 4, 4, 16, generator=g) / 16).to(DEV).to(bf)
    bias = (torch.randn(64, generator=g) * 0.1).to(DEV)
    y1 = torch.empty(N, H2, W2, 64, dtype=bf, device=DEV)
    call("retr_conv2d_fwd_out", ops.dcode(bf), ptr(xs), N, H2, W2, 16, ptr(w2), ptr(bias), None,
         ptr(y1), 64, 4, 4, 1, 2, 1, H2, W2, 1, ops._st())
    PH, PW = (H2 - 1) // 2 + 1, (W2 - 1) // 2 + 1
    ref = torch.empty(N, PH, PW, 64, dtype=bf, device=DEV)
    call("retr_maxpool3x3s2", ops.dcode(bf), ptr(y1), ptr(ref), N, H2, W2, 64, PH, PW, ops._st())
    y = torch.full((N, PH, PW, 64), float("nan"), dtype=bf, device=DEV)
    call("retr_stem_pool_fwd", ops.dcode(bf), ptr(xs), N, H2, W2, ptr(w2), ptr(bias), ptr(y), 64,
         ops._st())
    torch.cuda.synchronize()
    assert torch.equal(y, ref), (y.float() - ref.float()).abs().max()
    # and against fp32 torch (conv over the s2d image, pad 2, cropped to H2 x W2; pool)
    conv = F.conv2d(xs.float().permute(0, 3, 1, 2).cpu(), w2.float().permute(0, 3, 1, 2).cpu(),
                    padding=2)[:, :, :H2, :W2]
    tref = F.max_pool2d(torch.relu(conv + bias.cpu().view(1, -1, 1, 1)), 3, 2, 1)
    assert rel_err(y.permute(0, 3, 1, 2).float().cpu(), tref) < 1e-2


def test_conv_pack_cache_lives_on_the_spec():
    """Packed conv weights are cached on each ConvSpec (they die with the model): a dict keyed by
    id(spec) served a later model -- whose specs reused dead ids and whose tensors reused the
    same addresses -- the dead model's packed weights (intermittent test_gpu_optim failure)."""
    from tests.helpers import make_config
    from retr_amd.models.caption import build_model
    from retr_amd.models.utils import NestedTensor
    from retr_amd.synthetic import synthetic_images
    assert not hasattr(resnet.PACKS, "_d")
    model, _ = build_model(make_config())
    model.to(DEV).eval()
    img, mask = synthetic_images(1, 64, seed=3)
    with torch.no_grad():
        model(NestedTensor(img.to(DEV), mask.to(DEV)),
              torch.zeros(1, 16, dtype=torch.long, device=DEV),
              torch.zeros(1, 16, dtype=torch.bool, device=DEV))
    specs = [s for m in model.modules() if isinstance(getattr(m, "_runner", None),
                                                       resnet.BackboneRunner)
             for s in m._runner.specs]
    assert specs and all(s.pack is not None for s in specs)


@pytest.mark.parametrize("N,H,W,C1,C2,Co,s", [(2, 20, 20, 64, 64, 256, 1),
                                              (3, 7, 9, 64, 64, 256, 1),
                                              (1, 28, 28, 512, 1024, 2048, 1),
                                              (16, 160, 160, 64, 64, 256, 1),
                                              (2, 10, 10, 128, 256, 512, 2),
                                              (3, 5, 7, 256, 512, 1024, 2),
                                              (16, 80, 80, 128, 256, 512, 2)])
def test_conv1x1_fwd_cat(N, H, W, C1, C2, Co, s):
    """retr_conv1x1_fwd_cat (bottleneck conv3 + 1x1 downsample of stride s + residual + ReLU as
    one conv over [h2 | x[:, ::s, ::s]]) against fp32 torch, and against the unfused pair
    (downsample conv, then conv3 with its output as the residual: differs by that output's
    bf16 rounding).  H2 = s * H (even) or s * H - 1 (odd input rows, as torchvision's)."""
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(N * H * W + C2 + s)
    M = N * H * W
    H2, W2 = (s * H, s * W - (1 if s > 1 else 0))
    x1 = torch.randn(M, C1, generator=g).to(DEV, bf)
    x2 = torch.randn(N, H2, W2, C2, generator=g).to(DEV, bf)
    w1 = (torch.randn(Co, C1, generator=g) / math.sqrt(C1)).to(DEV, bf)
    w2 = (torch.randn(Co, C2, generator=g) / math.sqrt(C2)).to(DEV, bf)
    b1 = torch.randn(Co, generator=g).to(DEV)
    b2 = torch.randn(Co, generator=g).to(DEV)
    wcat = torch.cat([w1, w2], 1).contiguous()
    bcat = b1 + b2
    y = torch.full((M, Co), float("nan"), dtype=bf, device=DEV)
    call("retr_conv1x1_fwd_cat", ops.dcode(bf), ptr(x1), C1, ptr(x2), C2, N, H, W, H2, W2, s,
         ptr(wcat), ptr(bcat), ptr(y), Co, 1, ops._st())
    xs = x2[:, ::s, ::s, :].reshape(M, C2)
    ref = torch.relu(x1.float() @ w1.float().t() + xs.float() @ w2.float().t() + bcat)
    assert rel_err(y.float(), ref) < 1e-2
    yd = torch.empty(M, Co, dtype=bf, device=DEV)
    call("retr_conv2d_fwd", ops.dcode(bf), ptr(x2), N, H2, W2, C2, ptr(w2), ptr(b2), None,
         ptr(yd), Co, 1, 1, s, 0, 1, 0, ops._st())
    yu = torch.empty(M, Co, dtype=bf, device=DEV)
    call("retr_conv2d_fwd", ops.dcode(bf), ptr(x1), N, H, W, C1, ptr(w1), ptr(b1), ptr(yd),
         ptr(yu), Co, 1, 1, 1, 0, 1, 1, ops._st())
    torch.cuda.synchronize()
    assert rel_err(y.float(), yu.float()) < 1e-2
    assert torch.isfinite(y.float()).all()


@pytest.mark.parametrize("N,H,W,ds", [(2, 16, 32, False), (2, 24, 48, True), (1, 40, 16, False),
                                      (3, 8, 16, True)])
def test_bottleneck_s1_fused_equals_three_launches(N, H, W, ds):
    """retr_bottleneck_s1_fwd (the frozen layer1 block in one launch, h1 / h2 in LDS) equals the
    unfused path bitwise: conv1 + conv2 (retr_conv2d_fwd) and conv3 with the identity residual
    (retr_conv2d_fwd) or with the 1x1 downsample folded in (retr_conv1x1_fwd_cat)."""
    bf = torch.bfloat16
    cin = 64 if ds else 256
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + H + W + int(ds))
    x = torch.randn(N, H, W, cin, generator=g).to(DEV).to(bf)
    w1 = (torch.randn(64, cin, generator=g) / math.sqrt(cin)).to(DEV).to(bf)
    w2 = (torch.randn(64, 3, 3, 64, generator=g) / 24).to(DEV).to(bf)
    k3 = 64 + (cin if ds else 0)
    w3 = (torch.randn(256, k3, generator=g) / math.sqrt(k3)).to(DEV).to(bf)
    b1, b2, b3 = (torch.randn(c, generator=g).to(DEV) * 0.1 for c in (64, 64, 256))
    st = ops._st()
    # unfused
    h1 = torch.empty(N, H, W, 64, dtype=bf, device=DEV)
    h2 = torch.empty_like(h1)
    y0 = torch.empty(N, H, W, 256, dtype=bf, device=DEV)
    call("retr_conv2d_fwd", 1, ptr(x), N, H, W, cin, ptr(w1), ptr(b1), None, ptr(h1), 64, 1, 1,
         1, 0, 1, 1, st)
    call("retr_conv2d_fwd", 1, ptr(h1), N, H, W, 64, ptr(w2), ptr(b2), None, ptr(h2), 64, 3, 3,
         1, 1, 1, 1, st)
    if ds:
        call("retr_conv1x1_fwd_cat", 1, ptr(h2), 64, ptr(x), cin, N, H, W, H, W, 1, ptr(w3),
             ptr(b3), ptr(y0), 256, 1, st)
    else:
        call("retr_conv2d_fwd", 1, ptr(h2), N, H, W, 64, ptr(w3), ptr(b3), ptr(x), ptr(y0), 256,
             1, 1, 1, 0, 1, 1, st)
    y1 = torch.full_like(y0, float("nan"))
    call("retr_bottleneck_s1_fwd", 1, ptr(x), N, H, W, cin, ptr(w1), ptr(b1), ptr(w2), ptr(b2),
         ptr(w3), ptr(b3), int(ds), ptr(y1), st)
    torch.cuda.synchronize()
    assert torch.isfinite(y1.float()).all()
    assert torch.equal(y1, y0), (y1.float() - y0.float()).abs().max().item()
    # and against an fp32 reference of the same bf16 operands (rounding of h1 / h2 included)
    xf = x.float().permute(0, 3, 1, 2)
    r1 = torch.relu(F.conv2d(xf, w1.float().view(64, cin, 1, 1)) + b1.view(1, -1, 1, 1))
    r1 = r1.to(bf).float()
    r2 = torch.relu(F.conv2d(r1, w2.float().permute(0, 3, 1, 2), padding=1) + b2.view(1, -1, 1, 1))
    r2 = r2.to(bf).float()
    if ds:
        r3 = F.conv2d(torch.cat([r2, xf], 1), w3.float().view(256, k3, 1, 1)) + b3.view(1, -1, 1, 1)
    else:
        r3 = F.conv2d(r2, w3.float().view(256, 64, 1, 1)) + b3.view(1, -1, 1, 1) + xf
    assert rel_err(y1.permute(0, 3, 1, 2), torch.relu(r3)) < 1e-2


@pytest.mark.parametrize("B,H,Lq,Lk,hd,causal,masked,mode", [
    (16, 8, 400, 400, 32, False, True, 0), (16, 8, 128, 400, 32, False, True, 0),
    (16, 8, 128, 128, 32, True, False, 0), (2, 8, 130, 200, 64, False, True, 0),
    (3, 8, 100, 77, 32, False, True, 2), (3, 8, 100, 77, 32, True, True, 1)])
def test_attention_saved_dropout_bits_equal_rehash(B, H, Lq, Lk, hd, causal, masked, mode):
    """retr_attention_fwd_dm saves the dropout keep bits, retr_attention_bwd_dm reads them (the
    resident dq3 / dkdv3 kernels; the streaming backward, mode 1, ignores them): outputs, lse and
    all three gradients bitwise those of the re-hashing path, and the saved bits are the keep
    decisions (their density is 1 - p)."""
    g = torch.Generator(device="cpu").manual_seed(Lq * 5 + Lk)
    C, p = H * hd, 0.1
    bf = torch.bfloat16
    q, k, v, do = (torch.randn(B * L, C, generator=g).to(DEV).to(bf) for L in (Lq, Lk, Lk, Lq))
    kpm = None
    if masked:
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[:, Lk - Lk // 5:] = 1
        kpm = kpm.to(DEV)
    outs = []
    _lib.load().retr_tune(5, mode)
    try:
        for use in (False, True):
            dm = ops.attn_dmask(B, H, Lq, Lk, p, bf, hd, DEV) if use else None
            if dm is not None:
                dm.fill_(-1)
            o = torch.empty(B * Lq, C, dtype=bf, device=DEV)
            lse = torch.empty(B * H * Lq, device=DEV)
            ops.k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, causal, p, 99, lse, None, dm)
            dq, dk, dv = (torch.empty_like(t) for t in (q, k, v))
            ops.k_attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, hd, kpm, causal, p,
                                99, dm)
            torch.cuda.synchronize()
            outs.append((o, lse, dq, dk, dv))
    finally:
        _lib.load().retr_tune(5, 0)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    if causal:   # words of key tiles past a block's diagonal are never written
        return
    # keep-bit density over every (b, h): the effective seed includes the process's device step
    # seed, so one (b, h) of a small shape (7700 bits, sigma 0.0034) could land outside the bound
    nw = (Lk + 31) // 32
    words = dm.view(B * H, nw, Lq).cpu().numpy().astype(np.uint32)
    bits = np.unpackbits(words.view(np.uint8).reshape(B * H, nw, Lq, 4), axis=3,
                         bitorder="little")
    bits = bits.reshape(B * H, nw, Lq, 32).transpose(0, 2, 1, 3).reshape(B * H, Lq, nw * 32)
    bits = bits[:, :, :Lk]
    assert abs(bits.mean() - (1 - p)) < 0.005, bits.mean()


@pytest.mark.parametrize("B,H,Lq,Lk,hd,causal,masked,fs", [
    (16, 8, 400, 400, 32, False, True, 0), (16, 8, 128, 400, 32, False, False, 0),
    (16, 8, 128, 128, 32, True, False, 0), (3, 8, 100, 77, 32, False, True, 1),
    (3, 8, 100, 300, 32, True, True, 4), (2, 8, 130, 200, 64, False, True, 2),
    (2, 8, 200, 200, 64, True, True, 1)])
def test_attention_pregenerated_keep_bits(B, H, Lq, Lk, hd, causal, masked, fs):
    """Training forwards with saved dropout bits: attn_keep_bits_kernel writes every keep word
    and the streaming forward reads them (RETR_TUNE_ATTN_KEEPPRE 1, opt-in) instead of hashing
    per score (knob 0, the default: the forward writes the bits itself).  Outputs, log-sum-exp and
    every word the hashing forward writes are bitwise equal, on the unsplit and key-split
    kernels (fs: RETR_TUNE_ATTN_FSPLIT), ragged, causal and key-padded shapes, hd 32 / 64."""
    g = torch.Generator(device="cpu").manual_seed(Lq * 7 + Lk)
    C, p = H * hd, 0.1
    bf = torch.bfloat16
    q, k, v = (torch.randn(B * L, C, generator=g).to(DEV).to(bf) for L in (Lq, Lk, Lk))
    kpm = None
    if masked:
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[:, Lk - Lk // 5:] = 1
        kpm = kpm.to(DEV)
    outs = {}
    _lib.load().retr_tune(12, fs)
    try:
        for pre in (0, 1):
            _lib.load().retr_tune(26, pre)
            dm = ops.attn_dmask(B, H, Lq, Lk, p, bf, hd, DEV)
            dm.fill_(0)
            o = torch.empty(B * Lq, C, dtype=bf, device=DEV)
            lse = torch.empty(B * H * Lq, device=DEV)
            ops.k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, causal, p, 11, lse, None, dm)
            torch.cuda.synchronize()
            outs[pre] = (o, lse, dm)
    finally:
        _lib.load().retr_tune(26, 0)
        _lib.load().retr_tune(12, 0)
    (o1, l1, d1), (o0, l0, d0) = outs[1], outs[0]     # pregenerated, hashing forward
    assert torch.equal(o0, o1) and torch.equal(l0, l1)
    w = d0 != 0 if causal else torch.ones_like(d0, dtype=torch.bool)
    assert torch.equal(d0[w], d1[w])
    assert w.float().mean().item() > (0.2 if causal else 0.99)   # words the comparison covers


@pytest.mark.parametrize("B,H,Lq,Lk,hd,causal,masked", [
    (16, 8, 128, 400, 32, False, True), (16, 8, 128, 128, 32, True, False),
    (3, 8, 100, 77, 32, False, True), (3, 8, 100, 300, 32, True, True),
    (2, 8, 130, 200, 64, False, True), (2, 8, 200, 200, 64, True, True)])
def test_attention_forward_key_split(B, H, Lq, Lk, hd, causal, masked):
    """The key-split streaming forward (attn_fwd2s_kernel: 2 or 4 key parities per 32 queries,
    (m, l, O) merged through LDS in parity order) against the unsplit kernel: the dropout keep
    bits it saves are bitwise the same decisions, outputs and log-sum-exp agree to fp32 / bf16
    rounding, and each variant is deterministic (two runs bitwise equal)."""
    g = torch.Generator(device="cpu").manual_seed(Lq * 3 + Lk)
    C, p = H * hd, 0.1
    bf = torch.bfloat16
    q, k, v = (torch.randn(B * L, C, generator=g).to(DEV).to(bf) for L in (Lq, Lk, Lk))
    kpm = None
    if masked:
        kpm = torch.zeros(B, Lk, dtype=torch.uint8)
        kpm[:, Lk - Lk // 5:] = 1
        kpm = kpm.to(DEV)
    outs = {}
    try:
        for fs in (1, 2, 3, 4):
            _lib.load().retr_tune(12, fs)
            runs = []
            for _ in range(2):
                dm = ops.attn_dmask(B, H, Lq, Lk, p, bf, hd, DEV)
                dm.fill_(0)
                o = torch.empty(B * Lq, C, dtype=bf, device=DEV)
                lse = torch.empty(B * H * Lq, device=DEV)
                ops.k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, causal, p, 5, lse, None, dm)
                torch.cuda.synchronize()
                runs.append((o, lse, dm))
            for a, b in zip(*runs):
                assert torch.equal(a, b), fs
            outs[fs] = runs[0]
    finally:
        _lib.load().retr_tune(12, 0)
    o1, l1, d1 = outs[1]
    for fs in (2, 3, 4):
        o, lse, dm = outs[fs]
        if causal:   # a causal wave skips the key tiles past its own diagonal: fewer words
            w = dm != 0
            assert torch.equal(dm[w], d1[w]), fs
        else:
            assert torch.equal(dm, d1), fs
        assert (lse - l1).abs().max().item() < 1e-4, fs
        e = ((o.float() - o1.float()).norm() / o1.float().norm()).item()
        assert e < 5e-3, (fs, e)


@pytest.mark.parametrize("kind", ["fwd1x1", "dgrad1x1", "dgrad3x3s2", "ffn", "fwd1x1_k512",
                                  "dgrad1x1_k512"])
def test_shortk_single_stage_tiles_bitwise(kind):
    """Short-K wide GEMMs on the single-stage 64x64 tile (RETR_TUNE_SHORTK) and the large
    stride-2 dgrad phases on the single-stage 64x128 tile accumulate the same K-steps in the same
    order as the tiles they replaced: outputs bitwise equal with the rule on and off, and within
    bf16 rounding of fp32 torch.  (The *_k512 layer-4 shapes stay on their tiles either way:
    parity coverage for the 512-deep 1x1 convs.)"""
    g = torch.Generator(device="cpu").manual_seed(11)
    bf = torch.bfloat16
    outs, ref = [], None
    for off in (1, 0):
        _lib.load().retr_tune(14, off)
        try:
            if kind.startswith("fwd1x1"):   # 80x80x128 -> 512 + residual + ReLU (layer2 conv3)
                # or 20x20x512 -> 2048 (layer4 conv3, <= 8192 pixels)
                Nb, H, C, Co = (2, 80, 128, 512) if kind == "fwd1x1" else (4, 20, 512, 2048)
                if ref is None:
                    x = torch.randn(Nb, H, H, C, generator=g).to(DEV).to(bf)
                    w = (torch.randn(Co, C, generator=g) / math.sqrt(C)).to(DEV).to(bf)
                    b = torch.randn(Co, generator=g).to(DEV)
                    res = torch.randn(Nb, H, H, Co, generator=g).to(DEV).to(bf)
                    ref = torch.relu(x.float() @ w.float().t() + b + res.float())
                y = torch.empty(Nb, H, H, Co, dtype=bf, device=DEV)
                call("retr_conv2d_fwd", 1, ptr(x), Nb, H, H, C, ptr(w), ptr(b), ptr(res), ptr(y),
                     Co, 1, 1, 1, 0, 1, 1, ops._st())
            elif kind in ("dgrad1x1", "dgrad3x3s2", "dgrad1x1_k512"):
                # 80x80x512 <- 128 with the residual addend (layer2 conv3's data gradient), or
                # 160x160x128 <- 128 3x3 stride 2 (layer2.0 conv2: >= 64k pixels per phase)
                # or 20x20x2048 <- 512 (layer4 conv1's, K 512)
                Nb, H, C, Co, k, s_, p_ = {"dgrad1x1": (2, 80, 512, 128, 1, 1, 0),
                                           "dgrad1x1_k512": (4, 20, 2048, 512, 1, 1, 0),
                                           "dgrad3x3s2": (11, 160, 128, 128, 3, 2, 1)}[kind]
                OH = (H + 2 * p_ - k) // s_ + 1
                if ref is None:
                    w = torch.randn(Co, C, k, k, generator=g) / math.sqrt(C * k * k)
                    wp, wt, _, _, cp, _ = _pack(w.to(DEV), bf)
                    assert cp == C
                    weff = wp.float()[..., :C].permute(0, 3, 1, 2).cpu()
                    gy = torch.randn(Nb, Co, OH, OH, generator=g).to(bf).float()
                    add = (torch.randn(Nb, H, H, C, generator=g).to(bf)
                           if kind.startswith("dgrad1x1") else None)
                    xreq = torch.zeros(Nb, C, H, H, requires_grad=True)
                    F.conv2d(xreq, weff, stride=s_, padding=p_).backward(gy)
                    ref = xreq.grad.permute(0, 2, 3, 1).to(DEV)
                    if add is not None:
                        ref = ref + add.float().to(DEV)
                    gn = gy.permute(0, 2, 3, 1).contiguous().to(DEV).to(bf)
                    add_d = add.to(DEV) if add is not None else None
                y = torch.empty(Nb, H, H, C, dtype=bf, device=DEV)
                call("retr_conv2d_dgrad", 1, ptr(gn), Nb, H, H, C, ptr(wt), ptr(y), Co, k, k, s_,
                     p_, 1, ptr(add_d), None, ops._st())
            else:                     # encoder FFN expansion 6400 x 2048 x 256, bias + ReLU
                M, N, K = 6400, 2048, 256
                if ref is None:
                    x = torch.randn(M, K, generator=g).to(DEV).to(bf)
                    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV).to(bf)
                    b = torch.randn(N, generator=g).to(DEV)
                    ref = torch.relu(x.float() @ w.float().t() + b)
                y = torch.empty(M, N, dtype=bf, device=DEV)
                call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N, 0, M, N, K, 1,
                     None, 0, 0.0, 0, ops._st())
            torch.cuda.synchronize()
            outs.append(y)
        finally:
            _lib.load().retr_tune(14, 0)
    assert torch.equal(outs[0], outs[1])
    assert rel_err(outs[1].float(), ref) < 1e-2


@pytest.mark.parametrize("scale", [1.0, 2.0])
def test_fused_cross_entropy_matches_two_pass(scale):
    """Training-mode CrossEntropyLoss (bf16 logits): retr_ce_fwd_bwd writes lse, the loss and
    dlogits for dloss = 1 in one pass over the logits, retr_ce_bwd_rescale recomputes the
    gradient only for dloss != 1 -- against the two-pass kernels and fp32 torch."""
    from retr_amd.models.caption import CrossEntropyLoss
    g = torch.Generator(device="cpu").manual_seed(5)
    B, T, V, Vp = 4, 33, 30522, 30528
    store = (torch.randn(B, T, Vp, generator=g) * 3).to(DEV).to(torch.bfloat16)
    tgt = torch.randint(0, V, (B, T), generator=g).to(DEV)
    res = []
    try:
        for fused in (False, True):
            ops.FUSED_CE = fused
            x = store.clone().requires_grad_(True)
            loss = CrossEntropyLoss()(x[..., :V].permute(0, 2, 1), tgt)
            (loss * scale).backward()
            torch.cuda.synchronize()
            res.append((loss.detach().clone(), x.grad.detach().clone()))
    finally:
        ops.FUSED_CE = True
    (l0, g0), (l1, g1) = res
    ref = F.cross_entropy(store[..., :V].float().permute(0, 2, 1), tgt)
    assert abs(l1.item() - ref.item()) < 1e-4 * abs(ref.item())
    assert abs(l1.item() - l0.item()) < 1e-5 * abs(l0.item())
    assert torch.equal(g1[..., V:], torch.zeros_like(g1[..., V:]))
    e = ((g1.float() - g0.float()).norm() / g0.float().norm()).item()
    assert e < 1e-2, e


@pytest.mark.parametrize("dt,M,C,period", [(torch.bfloat16, 2048, 256, 128),
                                           (torch.float32, 6400, 256, 400),
                                           (torch.bfloat16, 100, 12, 7)])
def test_pos_grad_rows_in_order(dt, M, C, period):
    """retr_pos_grad (dpos[p] += sum of rows p, p + period, ... in row order; the 8-column
    vector kernel for C % 8 == 0, the scalar one otherwise) equals the in-order fp32 sum, and
    retr_pos_grad_set writes that sum."""
    g = torch.Generator(device="cpu").manual_seed(M + C)
    d = torch.randn(M, C, generator=g).to(dt)
    init = torch.randn(period, C, generator=g)
    dpos = init.clone().to(DEV)
    call("retr_pos_grad", ops.dcode(dt), ptr(d.to(DEV)), C, M, C, period, ptr(dpos), ops._st())
    torch.cuda.synchronize()
    df = d.float().numpy()
    s = np.zeros((period, C), dtype=np.float32)
    for m in range(M):
        s[m % period] += df[m]
    ref = init.numpy() + s
    assert np.array_equal(dpos.cpu().numpy(), ref)
    # overwrite mode (retr_pos_grad_set): the old contents (NaN here) are never read
    dset = torch.full((period, C), float("nan"), device=DEV)
    call("retr_pos_grad_set", ops.dcode(dt), ptr(d.to(DEV)), C, M, C, period, ptr(dset),
         ops._st())
    torch.cuda.synchronize()
    assert np.array_equal(dset.cpu().numpy(), np.float32(0) + s)


@pytest.mark.parametrize("case", ["ffn6400", "attn2048", "ragged"])
def test_wgrad_group_last_arriver_equals_slab_sum(case):
    """Grouped bf16 weight + bias gradients with the split-K reduction done by each output
    tile's last-arriving block inside the GEMM launch (RETR_TUNE_WGRAD_FUSED 1) against slabs +
    the separate slab_sum_group launch (knob 0, the default): bitwise equal (both add the slices in
    slice order), with the LayerNorm-style partial rows summed by the same launch's side
    blocks; repeated launches (tickets re-armed by the last arriver) stay bitwise identical."""
    from retr_amd import _lib
    shapes = {"ffn6400": [(6400, 256, 2048), (6400, 2048, 256)],
              "attn2048": [(2048, 256, 256), (2048, 512, 256), (6400, 256, 256),
                           (6400, 256, 256)],
              "ragged": [(1000, 200, 136), (777, 72, 64)]}[case]
    g = torch.Generator(device="cpu").manual_seed(len(case))
    items = []
    for i, (M, N, K) in enumerate(shapes):
        dy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        items.append([dy, x, M, N, K, i % 2 == 0])
    nparts, C = 37, 256
    parts = torch.randn(nparts * 2 * C, generator=g).to(DEV)
    outs = []
    try:
        for knob in (0, 1, 1, 1):
            _lib.load().retr_tune(17, knob)
            for acc in (False, True):
                run = []
                for dy, x, M, N, K, has_b in items:
                    dw = torch.randn(N, K, generator=torch.Generator().manual_seed(N + K)).to(DEV)
                    db = torch.randn(N, generator=torch.Generator().manual_seed(N)).to(DEV) \
                        if has_b else None
                    run.append((dy, x, dw, db, acc))
                gam = torch.randn(C, generator=torch.Generator().manual_seed(1)).to(DEV)
                bet = torch.randn(C, generator=torch.Generator().manual_seed(2)).to(DEV)
                extra = [(parts, 2 * C, nparts, C, gam, acc),
                         (parts[C:], 2 * C, nparts, C, bet, acc)]
                ops.k_linear_wgrad_group(run, extra)
                torch.cuda.synchronize()
                outs.append([t.clone() for it in run for t in it[2:4] if t is not None] +
                            [gam.clone(), bet.clone()])
    finally:
        _lib.load().retr_tune(17, 0)
    n = 2
    for k in range(1, 4):
        for a in range(n):
            ref, got = outs[a], outs[k * n + a]
            for r, t in zip(ref, got):
                assert torch.equal(r, t), (case, k, a)
    # and against fp32 torch (overwrite mode: dW = dY^T X, db = colsum dY; the LN rows)
    dy, x = items[0][0], items[0][1]
    assert rel_err(outs[2][0], dy.float().t() @ x.float()) < 1e-2
    assert rel_err(outs[2][1], dy.float().sum(0)) < 1e-2
    p2 = parts.view(nparts, 2, C)
    assert rel_err(outs[2][-2], p2[:, 0].sum(0)) < 1e-5
    assert rel_err(outs[2][-1], p2[:, 1].sum(0)) < 1e-5


@pytest.mark.parametrize("M", [6400, 2048, 1000])
def test_fused_ffn_equals_two_launch_path(M):
    """The fused FFN kernels (csrc/ffn.hip: retr_ffn_fwd / retr_ffn_bwd_data, the hidden chunk
    passed from the first GEMM's accumulators to the second GEMM's LDS operand) against the
    unfused launches (linear_fwd ReLU + linear_fwd_splitk, linear_dgrad gate + linear_dgrad_splitk)
    for a bf16 FFResidual block at d_model 256, F 2048, residual dropout 0.1: output, saved
    hidden activation and every gradient bitwise equal (same products, same order, the same
    F-split); and within bf16 rounding of an fp32 torch restatement
    (models/transformer_modules.py:6-11,77-97)."""
    from retr_amd.models.transformer_modules import FFResidual, feed_forward
    torch.manual_seed(M)
    mod = FFResidual(feed_forward(256, 2048), 256, dropout=0.1).to(DEV)
    with torch.no_grad():
        for p in mod.parameters():
            p.add_(torch.randn_like(p) * 0.02)
    x0 = torch.randn(M, 256, device=DEV)
    w_out = torch.randn(M, 256, device=DEV)
    res = []
    try:
        for fused in (False, True):
            ops.FUSE_FFN = fused
            ops._seed_state["ctr"] = 777
            mod.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            y = ops.ffn_block(mod, x, True, torch.bfloat16)
            (y * w_out).sum().backward()
            torch.cuda.synchronize()
            res.append((y.detach().clone(), x.grad.clone(),
                        {n: p.grad.clone() for n, p in mod.named_parameters()}))
    finally:
        ops.FUSE_FFN = False
    (y0, dx0, g0), (y1, dx1, g1) = res
    assert torch.equal(y0, y1)
    assert torch.equal(dx0, dx1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
    # fp32 restatement without dropout (eval) for scale
    ops.FUSE_FFN = True
    try:
        ye = ops.ffn_block(mod, x0, False, torch.bfloat16).float()
    finally:
        ops.FUSE_FFN = False
    ln = torch.nn.functional.layer_norm(x0, (256,), mod.norm.weight, mod.norm.bias, 1e-5)
    l1, l2 = mod.sublayer[0], mod.sublayer[2]
    ref = x0 + l2(torch.relu(l1(ln)))
    assert rel_err(ye - x0, ref - x0) < 2e-2


@pytest.mark.parametrize("tile", [0, 64, 128])
def test_wgrad_batch_matches_fp32_and_is_batching_invariant(tile):
    """retr_linear_wgrad_batch (the deferred weight gradients of whole transformer passes): every
    problem's dW = dY^T X and db = colsum dY (bias folded into the first column tile as an
    all-ones MFMA) against fp32 torch on the same bf16 operands, in overwrite and accumulate
    mode, plus LayerNorm-style partial-row sums in the same launch; and the bits do not depend
    on how the problems are batched (one launch of all vs three launches of subsets in another
    order) or on the tile (RETR_TUNE_WGRAD_TILE 64 / 128 / auto)."""
    from retr_amd import _lib
    # encoder block shapes (6400 tokens), decoder (2048), cross-attention K/V over the memory,
    # a ragged one (tokens and rows off every tile multiple)
    shapes = [(6400, 512, 256), (6400, 256, 256), (6400, 256, 256), (6400, 2048, 256),
              (6400, 256, 2048), (2048, 512, 256), (2048, 256, 256), (2048, 256, 256),
              (6400, 256, 256), (6400, 256, 256), (2048, 2048, 256), (2048, 256, 2048),
              (1000, 200, 136), (77, 72, 64)]
    g = torch.Generator(device="cpu").manual_seed(11)
    ops_ = []
    for i, (M, N, K) in enumerate(shapes):
        dy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        ops_.append((dy, x, i % 3 != 1))
    nparts, C = 53, 256
    parts = torch.randn(nparts * 2 * C, generator=g).to(DEV)

    def fresh(acc):
        run = []
        for k, (dy, x, has_b) in enumerate(ops_):
            N, K = dy.shape[1], x.shape[1]
            dw = torch.randn(N, K, generator=torch.Generator().manual_seed(k)).to(DEV)
            db = torch.randn(N, generator=torch.Generator().manual_seed(100 + k)).to(DEV) \
                if has_b else None
            run.append((dy, x, dw, db, acc))
        gam = torch.randn(C, generator=torch.Generator().manual_seed(1)).to(DEV)
        bet = torch.randn(C, generator=torch.Generator().manual_seed(2)).to(DEV)
        extra = [(parts, 2 * C, nparts, C, gam, acc), (parts[C:], 2 * C, nparts, C, bet, acc)]
        return run, extra

    def outs(run, extra):
        return [t.clone() for it in run for t in it[2:4] if t is not None] + \
               [e[4].clone() for e in extra]

    try:
        _lib.load().retr_tune(2, tile)          # RETR_TUNE_WGRAD_TILE
        res = {}
        for acc in (False, True):
            run, extra = fresh(acc)
            init = outs(run, extra)
            ops.k_linear_wgrad_batch(run, extra)
            torch.cuda.synchronize()
            got = outs(run, extra)
            res[acc] = got
            # fp32 references
            k = 0
            for dy, x, has_b in ops_:
                refw = dy.float().t() @ x.float()
                base = init[k] if acc else 0
                assert rel_err(got[k] - base, refw) < 2e-5, ("dw", dy.shape, x.shape, acc)
                k += 1
                if has_b:
                    base = init[k] if acc else 0
                    assert rel_err(got[k] - base, dy.float().sum(0)) < 2e-5, ("db", dy.shape)
                    k += 1
            p2 = parts.view(nparts, 2, C)
            for j in range(2):
                base = init[k + j] if acc else 0
                assert rel_err(got[k + j] - base, p2[:, j].sum(0)) < 1e-5
        # batching invariance: the same problems as three launches, reversed order
        run, extra = fresh(True)
        ops.k_linear_wgrad_batch(run[9:][::-1], extra)
        ops.k_linear_wgrad_batch(run[4:9])
        ops.k_linear_wgrad_batch(run[:4][::-1])
        torch.cuda.synchronize()
        for a, b in zip(res[True], outs(run, extra)):
            assert torch.equal(a, b)
    finally:
        _lib.load().retr_tune(2, 0)


def test_conv_wgrad_group_matches_fp32_and_single_path():
    """retr_conv2d_wgrad_group (the bf16 backbone's weight gradients, one grouped launch per
    loader kind with one K-slice length for all convs) + retr_conv_wgrad_unpack against fp32
    torch's conv2d weight gradient on the same bf16 operands (3x3 stride 1 / 2, dilated 3x3, 1x1
    stride 1 / 2, a ragged map), and against the per-conv retr_conv2d_wgrad path (same products,
    other slice boundaries: fp32 reassociation only)."""
    from torch.nn.grad import conv2d_weight
    from retr_amd import _lib
    # (Nb, H, W, C, Co, k, s, p, d)
    geos = [(4, 40, 40, 64, 64, 3, 1, 1, 1), (4, 40, 40, 64, 128, 3, 2, 1, 1),
            (2, 20, 20, 128, 64, 3, 1, 2, 2), (4, 40, 40, 128, 256, 1, 1, 0, 1),
            (4, 40, 40, 256, 128, 1, 1, 0, 1), (4, 40, 40, 64, 128, 1, 2, 0, 1),
            (3, 26, 18, 64, 64, 3, 1, 1, 1), (8, 80, 80, 64, 64, 1, 1, 0, 1)]
    g = torch.Generator().manual_seed(5)
    items = []
    for nb, h, w, c, co, k, s, p, d in geos:
        oh = (h + 2 * p - d * (k - 1) - 1) // s + 1
        ow = (w + 2 * p - d * (k - 1) - 1) // s + 1
        x = torch.randn(nb, h, w, c, generator=g).to(DEV, torch.bfloat16)
        dy = torch.randn(nb, oh, ow, co, generator=g).to(DEV, torch.bfloat16)
        items.append((x, dy, (nb, h, w, c, co, k, s, p, d)))
    n = len(items)
    arr = (_lib.ConvWgradDesc * n)()
    for i, (x, dy, (nb, h, w, c, co, k, s, p, d)) in enumerate(items):
        a = arr[i]
        a.dy, a.x = ptr(dy), ptr(x)
        a.Nb, a.H, a.W, a.C, a.Co, a.KH, a.KW, a.stride, a.pad, a.dil = nb, h, w, c, co, k, k, s, p, d
    call("retr_conv2d_wgrad_group_plan", 1, n, arr)
    assert all(arr[i].kind in (0, 1) for i in range(n))
    assert [arr[i].kind for i in range(n)] == [1, 1, 1, 0, 0, 1, 1, 0]
    slabs = []
    for i, (x, dy, (nb, h, w, c, co, k, s, p, d)) in enumerate(items):
        ws = torch.full((arr[i].splits, co, k * k * c), float("nan"), device=DEV)
        arr[i].ws = ptr(ws)
        slabs.append(ws)
    nbytes = int(_lib.load().retr_conv2d_wgrad_group_table_bytes(n)) + 512
    table = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    call("retr_conv2d_wgrad_group", 1, n, arr, ptr(table), nbytes, ops._st())
    for i, (x, dy, (nb, h, w, c, co, k, s, p, d)) in enumerate(items):
        got = torch.empty(co, c, k, k, device=DEV)
        call("retr_conv_wgrad_unpack", ptr(slabs[i]), None, ptr(got), co, c, c, k, k, 0,
             arr[i].splits, ops._st())
        ref = conv2d_weight(x.permute(0, 3, 1, 2).float(), (co, c, k, k),
                            dy.permute(0, 3, 1, 2).float(), stride=s, padding=p, dilation=d)
        assert rel_err(got, ref) < 1e-5, (geos[i], rel_err(got, ref))
        # the per-conv path (its own split plan)
        sp = int(_lib.load().retr_conv2d_wgrad_splits(1, nb, h, w, c, co, k, k, s, p, d))
        ws1 = torch.empty(sp, co, k * k * c, device=DEV)
        call("retr_conv2d_wgrad", 1, ptr(dy), ptr(x), nb, h, w, c, ptr(ws1), co, k, k, s, p, d,
             ops._st())
        one = torch.empty(co, c, k, k, device=DEV)
        call("retr_conv_wgrad_unpack", ptr(ws1), None, ptr(one), co, c, c, k, k, 0, sp, ops._st())
        assert rel_err(got, one) < 1e-6, (geos[i], rel_err(got, one))
    # every problem's slab sum + OIHW re-layout (+ a per-channel scale) in one grouped launch
    ua = (_lib.ConvUnpackDesc * n)()
    outs, scales = [], []
    for i, (x, dy, (nb, h, w, c, co, k, s, p, d)) in enumerate(items):
        sc = torch.rand(co, generator=g).to(DEV) + 0.5
        o = torch.full((co, c, k, k), float("nan"), device=DEV)
        u = ua[i]
        u.ws, u.scale, u.grad = ptr(slabs[i]), ptr(sc), ptr(o)
        u.Co, u.Ci, u.Cp, u.KH, u.KW, u.splits, u.accumulate = co, c, c, k, k, arr[i].splits, 0
        outs.append(o)
        scales.append(sc)
    nb2 = int(_lib.load().retr_conv_wgrad_unpack_group_table_bytes(n))
    utab = torch.empty((nb2 + 15) // 16 * 16, dtype=torch.uint8, device=DEV)
    call("retr_conv_wgrad_unpack_group", n, ua, ptr(utab), utab.numel(), ops._st())
    for i, (x, dy, (nb, h, w, c, co, k, s, p, d)) in enumerate(items):
        one = torch.empty(co, c, k, k, device=DEV)
        call("retr_conv_wgrad_unpack", ptr(slabs[i]), ptr(scales[i]), ptr(one), co, c, c, k, k,
             0, arr[i].splits, ops._st())
        assert rel_err(outs[i], one) < 1e-6, (geos[i], rel_err(outs[i], one))
    # round 5's kernel (RETR_TUNE_UNPACK_GRID -1: a block per 64 chunks, four waves' partial
    # sums through LDS; 37: the same with a capped grid) against the default row kernel (one
    # block per output channel, the four partials in registers): bitwise the same
    first = [o.clone() for o in outs]
    for knob in (-1, 37):
        for o in outs:
            o.fill_(float("nan"))
        try:
            _lib.load().retr_tune(28, knob)
            call("retr_conv_wgrad_unpack_group", n, ua, ptr(utab), utab.numel(), ops._st())
        finally:
            _lib.load().retr_tune(28, 0)
        for a, b in zip(first, outs):
            assert torch.equal(a, b), knob
    # accumulate mode: grad += scale * sum (the row kernel's staged and 16-byte paths)
    for i in range(n):
        ua[i].accumulate = 1
    base = [o.clone() for o in outs]
    call("retr_conv_wgrad_unpack_group", n, ua, ptr(utab), utab.numel(), ops._st())
    for a, b in zip(base, outs):
        assert torch.equal(b, a + a)
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,K", [(6400, 256, 2048), (2048, 256, 2048), (1000, 264, 1800)])
def test_splitk_fused_equals_slab_epilogue(M, N, K):
    """Split-K linears with the slice sum + epilogue done by each tile's last-arriving block
    (RETR_TUNE_SPLITK_FUSED 1, csrc/splitk_fused.hpp) against the slabs + separate
    slab-epilogue launch (knob 0): bitwise equal (both add the slices in slice order), forward
    with bias + residual + dropout (fp32 out) and data gradient with addend + ReLU gate (bf16
    out); repeated launches (tickets re-armed) stay bitwise identical."""
    bf = torch.bfloat16
    assert _lib.load().retr_linear_splits(1, M, N, K) > 1
    g = torch.Generator(device="cpu").manual_seed(M + K)
    x = torch.randn(M, K, generator=g).to(DEV).to(bf)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV).to(bf)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    dy = torch.randn(M, K, generator=g).to(DEV).to(bf)
    add = torch.randn(M, N, generator=g).to(DEV).to(bf)
    gate = torch.randn(M, N, generator=g).to(DEV).to(bf)
    wt = ops._TView(w.t().contiguous())
    outs = []
    try:
        for knob in (0, 1, 1, 1):
            _lib.load().retr_tune(18, knob)
            y = torch.full((M, N), float("nan"), device=DEV)
            ops.k_linear_fwd(x, w, b, y, res=res, drop_p=0.1, seed=91)
            dx = torch.full((M, N), float("nan"), dtype=bf, device=DEV)
            ops.k_linear_dgrad(dy, wt, dx, addend=add, gate=gate)
            torch.cuda.synchronize()
            outs.append((y, dx))
    finally:
        _lib.load().retr_tune(18, 0)
    for y, dx in outs[1:]:
        assert torch.equal(y, outs[0][0])
        assert torch.equal(dx, outs[0][1])
    ref = x.float() @ w.float().t() + b
    assert rel_err(outs[1][0], ref + res) < 0.5   # dropout applied: only a sanity bound


@pytest.mark.parametrize("nb,H,W,C,Co", [(16, 80, 80, 128, 128), (8, 40, 40, 256, 256),
                                         (4, 20, 20, 512, 512), (2, 26, 18, 64, 128),
                                         (3, 40, 40, 128, 256)])
def test_conv3x3_direct_matches_implicit_gemm_and_fp32(nb, H, W, C, Co):
    """The direct 3x3 stride-1 kernel (csrc/conv3x3.hip: input halo resident in LDS, one halo
    load per 64-channel chunk for all nine taps) against the implicit GEMM (RETR_TUNE_CONV3X3
    1) and fp32 torch on the same bf16 operands: forward (bias + ReLU, bf16 out) and data
    gradient (ReLU gate); ragged maps (26 x 18) and both tile shapes (16- and 20-pixel rows)."""
    import torch.nn.functional as F
    from torch.nn.grad import conv2d_input
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(H * W + C)
    x = torch.randn(nb, H, W, C, generator=g).to(DEV, bf)
    w = (torch.randn(Co, C, 3, 3, generator=g) / math.sqrt(9 * C)).to(DEV)
    b = torch.randn(Co, generator=g).to(DEV)
    wf = w.permute(0, 2, 3, 1).contiguous().to(bf)          # [Co][3][3][C] forward pack
    wt = w.permute(1, 2, 3, 0).contiguous().to(bf)          # [C][3][3][Co] dgrad pack
    dy = torch.randn(nb, H, W, Co, generator=g).to(DEV, bf)
    gate = torch.randn(nb, H, W, C, generator=g).to(DEV, bf)
    res = {}
    try:
        for knob in (2, 1):                     # 2: the direct kernel on every map (>= 16 wide)
            _lib.load().retr_tune(21, knob)
            y = torch.full((nb, H, W, Co), float("nan"), dtype=bf, device=DEV)
            call("retr_conv2d_fwd", 1, ptr(x), nb, H, W, C, ptr(wf), ptr(b), None, ptr(y), Co,
                 3, 3, 1, 1, 1, 1, ops._st())
            dx = torch.full((nb, H, W, C), float("nan"), dtype=bf, device=DEV)
            call("retr_conv2d_dgrad", 1, ptr(dy), nb, H, W, C, ptr(wt), ptr(dx), Co, 3, 3, 1, 1,
                 1, None, ptr(gate), ops._st())
            torch.cuda.synchronize()
            res[knob] = (y.float(), dx.float())
    finally:
        _lib.load().retr_tune(21, 0)
    xr = x.float().permute(0, 3, 1, 2)
    wr = wf.float().permute(0, 3, 1, 2)
    yref = torch.relu(F.conv2d(xr, wr, b, padding=1)).permute(0, 2, 3, 1)
    dxr = conv2d_input(xr.shape, wr, dy.float().permute(0, 3, 1, 2), padding=1)
    dxr = (dxr.permute(0, 2, 3, 1) * (gate.float() > 0))
    for knob in (2, 1):
        assert rel_err(res[knob][0], yref) < 1e-2, (knob, rel_err(res[knob][0], yref))
        assert rel_err(res[knob][1], dxr) < 1e-2, (knob, rel_err(res[knob][1], dxr))
    # same products in another fixed order: within bf16 rounding of the implicit GEMM
    assert rel_err(res[2][0], res[1][0]) < 5e-3
    assert rel_err(res[2][1], res[1][1]) < 5e-3


def test_conv3x3_direct_every_tile_variant():
    """Every RETR_TUNE_C3_TILE variant of the direct 3x3 kernel (tiles, 144 / 160-byte halo
    rows, two / three weight stages) against the implicit GEMM on a ragged map, forward and
    data gradient, and each variant bitwise stable over two launches (the weight-stage race of
    round 6 showed up as run-to-run differences)."""
    bf = torch.bfloat16
    nb, H, W, C, Co = 2, 22, 40, 128, 256
    g = torch.Generator().manual_seed(7)
    x = torch.randn(nb, H, W, C, generator=g).to(DEV, bf)
    wf = (torch.randn(Co, 3, 3, C, generator=g) / math.sqrt(9 * C)).to(DEV, bf)
    wt = (torch.randn(C, 3, 3, Co, generator=g) / math.sqrt(9 * Co)).to(DEV, bf)
    b = torch.randn(Co, generator=g).to(DEV)
    dy = torch.randn(nb, H, W, Co, generator=g).to(DEV, bf)
    gate = torch.randn(nb, H, W, C, generator=g).to(DEV, bf)

    def run():
        y = torch.full((nb, H, W, Co), float("nan"), dtype=bf, device=DEV)
        call("retr_conv2d_fwd", 1, ptr(x), nb, H, W, C, ptr(wf), ptr(b), None, ptr(y), Co, 3, 3,
             1, 1, 1, 1, ops._st())
        dx = torch.full((nb, H, W, C), float("nan"), dtype=bf, device=DEV)
        call("retr_conv2d_dgrad", 1, ptr(dy), nb, H, W, C, ptr(wt), ptr(dx), Co, 3, 3, 1, 1, 1,
             None, ptr(gate), ops._st())
        torch.cuda.synchronize()
        return y.float(), dx.float()

    lib = _lib.load()
    try:
        lib.retr_tune(21, 1)                    # the implicit GEMM
        ref = run()
        lib.retr_tune(21, 2)                    # the direct kernel on every map >= 16 wide
        for v in range(1, 14):
            lib.retr_tune(22, v)
            a, a2 = run(), run()
            for got, again, want in zip(a, a2, ref):
                assert torch.equal(got, again), v
                assert rel_err(got, want) < 5e-3, (v, rel_err(got, want))
    finally:
        lib.retr_tune(21, 0)
        lib.retr_tune(22, 0)


@pytest.mark.parametrize("M,N,K", [(6400, 2048, 256), (2048, 2048, 256), (1000, 1800, 192),
                                   (640, 1024, 128)])
def test_panel_gemm_equals_tile_gemm(M, N, K):
    """Short-reduction wide-output linears on the resident-A panel kernel (csrc/panel.hpp,
    RETR_TUNE_PANEL 1, opt-in) against the 64x64 gemm2 tile (knob 0, the default): bitwise equal (same MFMA chain
    per output), forward with bias + ReLU (bf16 out) and the ReLU-gated data gradient with the
    weight both as W^T (K-contiguous) and as W read transposed; ragged M and N; vs fp32 torch."""
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV).to(bf)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV).to(bf)
    b = torch.randn(N, generator=g).to(DEV)
    dy = torch.randn(M, K, generator=g).to(DEV).to(bf)            # dX[M][N] = dY[M][K] W2[K][N]
    w2 = (torch.randn(K, N, generator=g) / math.sqrt(K)).to(DEV).to(bf)
    gate = torch.randn(M, N, generator=g).to(DEV).to(bf)
    outs = {}
    try:
        for knob in (0, 1):
            _lib.load().retr_tune(23, knob)
            y = torch.full((M, N), float("nan"), dtype=bf, device=DEV)
            ops.k_linear_fwd(x, w, b, y, relu=1)
            d1 = torch.full((M, N), float("nan"), dtype=bf, device=DEV)
            ops.k_linear_dgrad(dy, w2.t().contiguous(), d1, gate=gate)       # W^T stored [N][K]
            d2 = torch.full((M, N), float("nan"), dtype=bf, device=DEV)
            ops.k_linear_dgrad(dy, ops._TView(w2), d2, gate=gate)            # W [K][N] transposed
            torch.cuda.synchronize()
            outs[knob] = (y, d1, d2)
    finally:
        _lib.load().retr_tune(23, 0)
    for a, c in zip(outs[1], outs[0]):
        assert torch.equal(a, c)
    ref = torch.relu(x.float() @ w.float().t() + b)
    assert rel_err(outs[1][0].float(), ref) < 1e-2
    dref = (dy.float() @ w2.float()) * (gate.float() > 0)
    assert rel_err(outs[1][1].float(), dref) < 1e-2
    assert torch.equal(outs[1][1], outs[1][2])


@pytest.mark.parametrize("M,N,K,period,plain,with_pos,drop", [
    (6400, 256, 2048, 400, True, True, 0.1), (2048, 256, 2048, 128, True, True, 0.1),
    (2048, 256, 2048, 0, True, False, 0.0), (1000, 256, 1536, 77, False, True, 0.1),
    (700, 512, 2048, 35, True, True, 0.1)])
def test_splitk_linear_with_next_layernorm(M, N, K, period, plain, with_pos, drop):
    """retr_linear_fwd_splitk_ln: the split-K down-projection (bias, dropout, fp32 residual)
    whose slab epilogue also writes LN(out) / LN(out) + pos[row % period], mean and rstd --
    bitwise equal to the split-K linear followed by retr_layernorm_fwd (the same slab-sum
    order, epilogue arithmetic and ln_fwd4 statistics), and LN within bf16 rounding of fp32
    torch."""
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV).to(bf)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV).to(bf)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    gam = (1 + 0.1 * torch.randn(N, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(N, generator=g)).to(DEV)
    pos = torch.randn(max(period, 1), N, generator=g).to(DEV) if with_pos else None
    assert ops._splits(bf, M, N, K) > 1
    outs = []
    for fused in (True, False):
        y = torch.full((M, N), float("nan"), device=DEV)
        ly = torch.full((M, N), float("nan"), dtype=bf, device=DEV) if plain else None
        ly2 = torch.full((M, N), float("nan"), dtype=bf, device=DEV) if with_pos else None
        mean = torch.empty(M, device=DEV)
        rstd = torch.empty(M, device=DEV)
        if fused:
            ops.k_linear_fwd(x, w, b, y, res=res, drop_p=drop, seed=3,
                             ln=(gam, bet, 1e-5, ly, ly2, pos, period, mean, rstd))
        else:
            ops.k_linear_fwd(x, w, b, y, res=res, drop_p=drop, seed=3)
            ly_, ly2_, mean_, rstd_ = ops._ln_fwd(y, gam, bet, 1e-5, bf, pos, period, plain,
                                                  with_pos)
            ly, ly2, mean, rstd = ly_, ly2_, mean_, rstd_
        torch.cuda.synchronize()
        outs.append((y, ly, ly2, mean, rstd))
    for a, c in zip(*outs):
        assert (a is None) == (c is None)
        if a is not None:
            assert torch.equal(a, c)
    y, ly, ly2, mean, rstd = outs[0]
    ref = torch.nn.functional.layer_norm(y, (N,), gam, bet, 1e-5)
    if plain:
        assert rel_err(ly.float(), ref) < 1e-2
    if with_pos:
        rows = torch.arange(M, device=DEV) % period
        assert rel_err(ly2.float(), ref + pos[rows]) < 1e-2
    if drop == 0.0:
        yref = x.float() @ w.float().t() + b + res
        assert rel_err(y, yref) < 1e-2


@pytest.mark.parametrize("n,acc,ld_pad", [(12, 1, 0), (12, 0, 0), (17, 1, 0), (3, 1, 8), (1, 0, 0)])
def test_pos_grad_multi_equals_per_item_launches(n, acc, ld_pad):
    """retr_pos_grad_multi (the decoder blocks' query-position gradients in one launch) against
    one retr_pos_grad per item in the same order (the first retr_pos_grad_set when not
    accumulating): bitwise equal, including more than 16 items (two launches) and row strides
    wider than C."""
    import ctypes
    from retr_amd import _lib as L
    T, B, C = 128, 16, 256
    g = torch.Generator(device="cpu").manual_seed(n * 7 + acc)
    items = [torch.randn(B * T, C + ld_pad, generator=g).to(DEV).to(torch.bfloat16)
             for _ in range(n)]
    init = torch.randn(T, C, generator=g).to(DEV)
    a = init.clone()
    for i, d in enumerate(items):
        name = "retr_pos_grad" if (acc or i > 0) else "retr_pos_grad_set"
        L.call(name, 1, L.ptr(d), d.stride(0), B * T, C, T, L.ptr(a), L.stream())
    b = init.clone()
    arr = (L.PosItem * n)()
    for i, d in enumerate(items):
        arr[i].d, arr[i].ld, arr[i].M = L.ptr(d), d.stride(0), B * T
    L.call("retr_pos_grad_multi", 1, n, arr, C, T, L.ptr(b), acc, L.stream())
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    ref = (init if acc else torch.zeros_like(init)) + sum(
        d[:, :C].float().view(B, T, C).sum(0) for d in items)
    assert rel_err(b, ref) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,kind", [(2048, 256, "fwd_res"), (6400, 256, "fwd_res"),
                                      (2048, 256, "fwd_relu"), (1000, 200, "fwd_res"),
                                      (2048, 256, "dgrad"), (6400, 256, "dgrad_t"),
                                      (777, 256, "dgrad")])
def test_linear_k256_all_steps_at_once_equals_loop(M, N, kind):
    """K = 256 linears on few output tiles: gemm_short_kernel (every K-step fetched at once,
    RETR_TUNE_LIN_K256 = 0 / 2) gives the bits of gemm_kernel's double-buffered loop (1), and
    both match an fp32 reference (ragged M / N included)."""
    bf, K, lib = torch.bfloat16, 256, _lib.load()
    g = torch.Generator(device=DEV).manual_seed(M + N)
    outs = []
    try:
        for knob in (1, 0):
            lib.retr_tune(33, knob)
            if kind.startswith("fwd"):
                x = torch.randn(M, K, device=DEV, generator=g).to(bf) if not outs else x
                w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).to(bf) if not outs else w
                b = torch.randn(N, device=DEV, generator=g) if not outs else b
                res = torch.randn(M, N, device=DEV, generator=g) if not outs else res
                y = torch.zeros(M, N, device=DEV)
                relu = int(kind == "fwd_relu")
                call("retr_linear_fwd", 1, ptr(x), K, ptr(w), K, ptr(b), ptr(y), N, 1, M, N, K,
                     relu, None if relu else ptr(res), N, 0.0, 0, _lib.stream())
                ref = x.float() @ w.float().t() + b
                ref = torch.relu(ref) if relu else ref + res
            else:
                # dX[M][K'] = dY[M][N'] W (reduction over N' = 256), ReLU gate + bf16 addend
                Kout = N
                dy = torch.randn(M, K, device=DEV, generator=g).to(bf) if not outs else dy
                wt = (torch.randn(K, Kout, device=DEV, generator=g) * 0.05).to(bf) if not outs else wt
                gate = torch.randn(M, Kout, device=DEV, generator=g).to(bf) if not outs else gate
                add = torch.randn(M, Kout, device=DEV, generator=g).to(bf) if not outs else add
                y = torch.zeros(M, Kout, device=DEV, dtype=bf)
                if kind == "dgrad_t":    # W^T stored [K'][N'] (w_trans 1)
                    wk = wt.t().contiguous()
                    call("retr_linear_dgrad", 1, ptr(dy), K, ptr(wk), K, ptr(y), Kout, 0, M, K,
                         Kout, ptr(add), 0, Kout, ptr(gate), Kout, 1, _lib.stream())
                else:
                    call("retr_linear_dgrad", 1, ptr(dy), K, ptr(wt), Kout, ptr(y), Kout, 0, M, K,
                         Kout, ptr(add), 0, Kout, ptr(gate), Kout, 0, _lib.stream())
                ref = (dy.float() @ wt.float() + add.float()) * (gate.float() > 0)
            torch.cuda.synchronize()
            outs.append(y.clone())
    finally:
        lib.retr_tune(33, 0)
    assert torch.equal(outs[0], outs[1])
    err = (outs[1].float() - ref).abs().max().item()
    assert err < 0.05 * max(1.0, ref.abs().max().item()), err
