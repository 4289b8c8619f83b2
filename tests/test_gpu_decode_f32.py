"""Fused decode step of the fp32 parity mode (csrc/decode_f32.hip, round 6) against plain
PyTorch fp32 references of the same ops, and the fused step against the per-op fp32 step on the
cfg5 model (eval_utils/decode.py:53-81 in KV-cache form).  The ids of the fused step are pinned
to the CPU oracle by tests/test_gpu_configs.py (test_cfg5_greedy_fp32_*: the default fp32 decode
path is this one)."""
import math

import pytest
import torch
import torch.nn.functional as F

from retr_amd import ops
from retr_amd._lib import call, ptr
from retr_amd.models.utils import NestedTensor

pytestmark = pytest.mark.gpu
DEV = "cuda"
C, H, HD = 256, 8, 32
TOL = 2e-6          # fp32, summation order only


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _g(seed):
    return torch.Generator().manual_seed(seed)


def _rn(*shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


def _mha_row(q, K, V, mask=None):
    """q [H, hd] (scaled) over keys K / V [L, H, hd] -> [H * hd] (fp64 reference)."""
    q, K, V = q.double(), K.double(), V.double()
    s = torch.einsum("hd,lhd->hl", q, K)
    if mask is not None:
        s = s.masked_fill(mask[None], float("-inf"))
    return torch.einsum("hl,lhd->hd", torch.softmax(s, -1), V).reshape(-1)


@pytest.mark.parametrize("i,beam,embed", [(0, False, True), (5, False, False),
                                          (77, True, False), (200, False, False)])
def test_dec_self_f32_matches_torch(i, beam, embed):
    """retr_dec_self_f32: prologue (FFN slabs + residual, or the token embedding + its LN), LN1
    (+ qpos), the head's q | k | v, cache append (row r, step i), attention over keys 0..i (beam
    ancestry), per-head partial out-projections -- against fp64 torch."""
    R, T, F_, V = 10, 256, 512, 50
    nslab = F_ // 64
    g = _g(100 + i)
    win, bin_ = _rn(3 * C, C, g=g, scale=0.06), _rn(3 * C, g=g)
    wo = _rn(C, C, g=g, scale=0.06)
    kc, vc = _rn(R * T, C, g=g), _rn(R * T, C, g=g)
    kc0, vc0 = kc.clone(), vc.clone()
    x, slabs, b2 = _rn(R, C, g=g), _rn(nslab, R, C, g=g, scale=0.3), _rn(C, g=g)
    tok = torch.randint(0, V, (R,), generator=g).to(DEV)
    word = _rn(V, C, g=g)
    ge, be = (torch.rand(C, generator=g) + 0.5).to(DEV), _rn(C, g=g, scale=0.1)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), _rn(C, g=g, scale=0.1)
    qpos = _rn(C, g=g)
    anc = None
    if beam:
        anc = torch.randint(0, R, (R, T), generator=g, dtype=torch.int32).to(DEV)
    slab = torch.empty(H, R, C, device=DEV)
    xout = torch.empty(R, C, device=DEV)
    pro = ((None, None, 0, None, ptr(tok), ptr(word), ptr(ge), ptr(be), 1e-12) if embed else
           (ptr(x), ptr(slabs), nslab, ptr(b2), None, None, None, None, 0.0))
    call("retr_dec_self_f32", R, C, H, ptr(win), ptr(bin_), ptr(kc), ptr(vc), i, T, ptr(anc),
         ptr(wo), ptr(slab), *pro, ptr(gamma), ptr(beta), 1e-5, ptr(qpos), ptr(xout), ops._st())
    torch.cuda.synchronize()
    d = lambda t: t.double()                                      # noqa: E731
    if embed:
        xr = F.layer_norm(d(word[tok] + qpos), (C,), d(ge), d(be), 1e-12)
    else:
        xr = d(x) + (d(slabs).sum(0) + d(b2))
    assert _rel(xout, xr) < TOL
    n = F.layer_norm(xr, (C,), d(gamma), d(beta), 1e-5)
    qkv_in = [n + d(qpos), n + d(qpos), n]
    q = qkv_in[0] @ d(win[:C]).t() + d(bin_[:C])
    k = qkv_in[1] @ d(win[C:2 * C]).t() + d(bin_[C:2 * C])
    v = qkv_in[2] @ d(win[2 * C:]).t() + d(bin_[2 * C:])
    kcv, vcv = kc.view(R, T, C), vc.view(R, T, C)
    assert _rel(kcv[:, i], k) < TOL and _rel(vcv[:, i], v) < TOL
    other = torch.ones(T, dtype=torch.bool)
    other[i] = False
    assert torch.equal(kcv[:, other], kc0.view(R, T, C)[:, other])   # only row i written
    ref = torch.empty(H, R, C, dtype=torch.float64)
    for r in range(R):
        rows = [int(anc[r, j]) if beam else r for j in range(i)]
        K = torch.stack([d(kc0.view(R, T, C)[rows[j], j]) for j in range(i)] + [k[r]]) \
            if i else k[r][None]
        Vv = torch.stack([d(vc0.view(R, T, C)[rows[j], j]) for j in range(i)] + [v[r]]) \
            if i else v[r][None]
        o = _mha_row((q[r] / math.sqrt(HD)).view(H, HD), K.view(-1, H, HD), Vv.view(-1, H, HD))
        for h in range(H):
            ref[h, r] = (o[h * HD:(h + 1) * HD] @ d(wo[:, h * HD:(h + 1) * HD]).t()).cpu()
    assert _rel(slab, ref) < 1e-5


@pytest.mark.parametrize("Lk,kv_group", [(37, 1), (196, 5), (300, 2)])
def test_dec_cross_f32_matches_torch(Lk, kv_group):
    """retr_dec_cross_f32: ordered head-partial sum + residual + LN2 + pos, the head's cross
    query, masked attention over the memory of the row's image, partial out-projection."""
    R = 10
    g = _g(Lk)
    slab_in, x, bo = _rn(H, R, C, g=g, scale=0.3), _rn(R, C, g=g), _rn(C, g=g)
    gamma, beta, pos = (torch.rand(C, generator=g) + 0.5).to(DEV), _rn(C, g=g), _rn(C, g=g)
    wq, bq, wo = _rn(C, C, g=g, scale=0.06), _rn(C, g=g), _rn(C, C, g=g, scale=0.06)
    nb = R // kv_group
    K, V = _rn(nb * Lk, C, g=g), _rn(nb * Lk, C, g=g)
    kpm = torch.zeros(nb, Lk, dtype=torch.uint8)
    kpm[0, Lk - 7:] = 1
    kpm = kpm.to(DEV)
    xo, slab = torch.empty(R, C, device=DEV), torch.empty(H, R, C, device=DEV)
    call("retr_dec_cross_f32", R, C, H, ptr(slab_in), ptr(x), ptr(bo), ptr(xo), ptr(gamma),
         ptr(beta), 1e-5, ptr(pos), ptr(wq), ptr(bq), ptr(K), ptr(V), Lk, kv_group, ptr(kpm),
         ptr(wo), ptr(slab), ops._st())
    torch.cuda.synchronize()
    d = lambda t: t.double()                                      # noqa: E731
    xr = d(x) + (d(slab_in).sum(0) + d(bo))
    assert _rel(xo, xr) < TOL
    qin = F.layer_norm(xr, (C,), d(gamma), d(beta), 1e-5) + d(pos)
    q = (qin @ d(wq).t() + d(bq)) / math.sqrt(HD)
    ref = torch.empty(H, R, C, dtype=torch.float64)
    for r in range(R):
        b = r // kv_group
        o = _mha_row(q[r].view(H, HD), d(K[b * Lk:(b + 1) * Lk]).view(Lk, H, HD),
                     d(V[b * Lk:(b + 1) * Lk]).view(Lk, H, HD), kpm[b].bool())
        for h in range(H):
            ref[h, r] = (o[h * HD:(h + 1) * HD] @ d(wo[:, h * HD:(h + 1) * HD]).t()).cpu()
    assert _rel(slab, ref) < 1e-5


@pytest.mark.parametrize("R", [7, 64])
def test_dec_ffn_f32_and_rows_match_torch(R):
    """retr_dec_ffn_f32 (head-partial sum + residual + LN3, FFN over 64 hidden units per block,
    exact-f32 MFMA) and retr_dec_rows_f32 (slab sum + residual + final LN) against fp64 torch."""
    F_ = 2048
    g = _g(R)
    x, hslab, bo = _rn(R, C, g=g), _rn(H, R, C, g=g, scale=0.3), _rn(C, g=g)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), _rn(C, g=g)
    w1, b1 = _rn(F_, C, g=g, scale=0.06), _rn(F_, g=g, scale=0.1)
    w2, b2 = _rn(C, F_, g=g, scale=0.02), _rn(C, g=g)
    xo = torch.empty(R, C, device=DEV)
    slabs = torch.empty(F_ // 64, R, C, device=DEV)
    call("retr_dec_ffn_f32", ptr(x), ptr(hslab), H, ptr(bo), ptr(gamma), ptr(beta), 1e-5,
         ptr(xo), R, C, ptr(w1), ptr(b1), ptr(w2), F_, ptr(slabs), ops._st())
    x2, n = torch.empty(R, C, device=DEV), torch.empty(R, C, device=DEV)
    call("retr_dec_rows_f32", ptr(xo), ptr(slabs), F_ // 64, ptr(b2), R, C, ptr(x2), ptr(gamma),
         ptr(beta), 1e-5, ptr(n), ops._st())
    torch.cuda.synchronize()
    d = lambda t: t.double()                                      # noqa: E731
    xr = d(x) + (d(hslab).sum(0) + d(bo))
    assert _rel(xo, xr) < TOL
    h = torch.relu(F.layer_norm(xr, (C,), d(gamma), d(beta), 1e-5) @ d(w1).t() + d(b1))
    ref_slabs = torch.stack([h[:, j:j + 64] @ d(w2[:, j:j + 64]).t() for j in range(0, F_, 64)])
    assert _rel(slabs, ref_slabs) < 1e-5
    ref_x2 = xr + (ref_slabs.sum(0) + d(b2))
    assert _rel(x2, ref_x2) < 1e-5
    assert _rel(n, F.layer_norm(ref_x2, (C,), d(gamma), d(beta), 1e-5)) < 1e-5


def test_fused_f32_step_matches_per_op_step_cfg5():
    """The fused fp32 step (three launches per decoder layer) against the per-op fp32 step on the
    cfg5 model: first-step logits to fp32 summation order, greedy ids and beam-5 ids equal, the
    hipGraph replay bitwise equal to eager launches."""
    from bench import build, cfg5
    from retr_amd.eval_utils import decode as dec
    from retr_amd.synthetic import synthetic_images
    model, _ = build(cfg5("fp32"), DEV)
    model.eval()
    B, T = 16, 128
    img, mask = synthetic_images(B, 224, seed=21, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    fused = dec.IncrementalGreedy(model, fused=True)
    ids_f = fused(s, T, 101, 102)
    st = next(v for k, v in model._retr_decode_states.items() if k[0] == "IncrementalGreedy" and k[-1])
    assert fused._fusable_f32(st) and st.hslab is not None
    old = dec.DEC_F32_FUSED
    try:
        dec.DEC_F32_FUSED = False
        plain = dec.IncrementalGreedy(model, fused=True)      # same state key: per-op step
        assert not plain._fusable_f32(st)
        ids_p = plain(s, T, 101, 102)
        with torch.no_grad():
            plain._reset(st, 101)
            plain._step(st, 0, 102)
            lp = st.logits.float().clone()
        model._retr_decode_states = {}
        ids_bp = dec.IncrementalBeam(model, 5)(s, T, 101, 102)
    finally:
        dec.DEC_F32_FUSED = old
    model._retr_decode_states = {}
    fused = dec.IncrementalGreedy(model, fused=True)
    ids_f2 = fused(s, T, 101, 102)
    st = next(v for k, v in model._retr_decode_states.items() if k[0] == "IncrementalGreedy" and k[-1])
    with torch.no_grad():
        fused._reset(st, 101)
        fused._step(st, 0, 102)
        lf = st.logits.float().clone()
    assert _rel(lf, lp) < 1e-5
    assert torch.equal(ids_f, ids_f2)
    assert torch.equal(ids_f, ids_p)
    ids_e = dec.IncrementalGreedy(model, use_graphs=False, fused=True)(s, T, 101, 102)
    assert torch.equal(ids_f, ids_e)
    ids_bf = dec.IncrementalBeam(model, 5)(s, T, 101, 102)
    # beam search ranks sums of log-probabilities over 5 x 30522 candidates per image and step:
    # fp32 summation-order differences (~1e-6) can flip a near-tie there, after which an image's
    # beams legitimately diverge -- most images must still agree token for token
    agree = (ids_bf == ids_bp).all(1).float().mean().item()
    assert agree >= 0.5, agree


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_split_batch_decode_equals_one_group(dtype):
    """DEC_SPLIT: the batch decoded as two independent row groups on concurrent streams of one
    graph gives the one-group decoder's ids token for token -- with an EOS that ends rows at
    different steps (each group writes every column, the batch ends at the last group's
    all-finished step and the later columns are cleared) and with one no row emits."""
    from bench import build, cfg5
    from retr_amd.eval_utils import decode as dec
    from retr_amd.synthetic import synthetic_images
    model, _ = build(cfg5(dtype), DEV)
    model.eval()
    B, T = 32, 128
    img, mask = synthetic_images(B, 224, seed=31, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    old = dec.DEC_SPLIT
    try:
        dec.DEC_SPLIT = 1
        probe = dec.IncrementalGreedy(model)(s, T, 101, 102)
        # an EOS that some rows emit early and others late / never
        vals, counts = torch.unique(probe[:, 2:12], return_counts=True)
        eos = int(vals[counts.argmax()])
        for e in (eos, 102):
            dec.DEC_SPLIT = 1
            ids1 = dec.IncrementalGreedy(model)(s, T, 101, e)
            dec.DEC_SPLIT = 2
            g2 = dec.IncrementalGreedy(model)
            assert g2._split(B) == 2
            ids2 = g2(s, T, 101, e)
            assert torch.equal(ids1, ids2), (e, (ids1 != ids2).nonzero()[:5].tolist())
            ids2b = g2(s, T, 101, e)                 # replayed graphs
            assert torch.equal(ids1, ids2b)
    finally:
        dec.DEC_SPLIT = old
        model._retr_decode_states = {}
