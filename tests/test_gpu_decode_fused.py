"""Fused incremental-decode kernels (csrc/decode.hip) against plain PyTorch fp32 references of
the same ops on the same bf16 operands, and the fused decode step against the unfused one on
the cfg5 model (eval_utils/decode.py:53-81 in KV-cache form)."""
import math

import pytest
import torch
import torch.nn.functional as F

from retr_amd import _lib, ops
from retr_amd._lib import call, ptr
from retr_amd.models.utils import NestedTensor

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _g(seed):
    return torch.Generator().manual_seed(seed)


@pytest.mark.parametrize("R", [5, 64, 70])
def test_dec_rows_and_gemm_segments(R):
    """dec_rows (ordered slab reduce + residual + LN (+pos)) feeding dec_gemm's three routed
    segments (q | k cache row i | v cache row i), and the head's single ReLU segment."""
    C, T, i, ns = 256, 12, 7, 5
    g = _g(R)
    x = torch.randn(R, C, generator=g).to(DEV)
    slabs = torch.randn(ns, R, C, generator=g).to(DEV)
    b2 = torch.randn(C, generator=g).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    pos = torch.randn(C, generator=g).to(DEV)
    xo = torch.empty(R, C, device=DEV)
    n = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
    npos = torch.empty_like(n)
    call("retr_dec_rows", ptr(x), ptr(slabs), ns, ptr(b2), R, C, ptr(xo), ptr(gamma), ptr(beta),
         1e-12, ptr(pos), ptr(n), ptr(npos), ops._st())
    ref_x = x + (slabs.sum(0) + b2)
    assert _rel(xo, ref_x) < 1e-6
    ln = F.layer_norm(ref_x, (C,), gamma, beta, 1e-12)
    assert _rel(n.float(), ln) < 1e-2 and _rel(npos.float(), ln + pos) < 1e-2
    w = (torch.randn(3 * C, C, generator=g) / 16).to(DEV).bfloat16()
    b = torch.randn(3 * C, generator=g).to(DEV)
    q = torch.zeros(R, C, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(R * T, C, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    call("retr_dec_gemm", ptr(n), ptr(npos), R, C, ptr(w), ptr(b), 3 * C, ptr(q), C, 1,
         ptr(kc) + 2 * i * C, T * C, 1, ptr(vc) + 2 * i * C, T * C, 0, C, 0, ops._st())
    wf = w.float()
    assert _rel(q.float(), npos.float() @ wf[:C].t() + b[:C]) < 1e-2
    assert _rel(kc.view(R, T, C)[:, i].float(), npos.float() @ wf[C:2 * C].t() + b[C:2 * C]) < 1e-2
    assert _rel(vc.view(R, T, C)[:, i].float(), n.float() @ wf[2 * C:].t() + b[2 * C:]) < 1e-2
    others = torch.ones(T, dtype=torch.bool)
    others[i] = False
    assert torch.count_nonzero(kc.view(R, T, C)[:, others]) == 0      # only row i written
    h = torch.empty(R, 512, dtype=torch.bfloat16, device=DEV)
    w1 = (torch.randn(512, C, generator=g) / 16).to(DEV).bfloat16()
    b1 = torch.randn(512, generator=g).to(DEV)
    call("retr_dec_gemm", ptr(n), None, R, C, ptr(w1), ptr(b1), 512, ptr(h), 512, 0, None, 0, 0,
         None, 0, 0, 512, 1, ops._st())
    assert _rel(h.float(), torch.relu(n.float() @ w1.float().t() + b1)) < 1e-2


def _attn_ref(qrow, K, V, mask, scale):
    """one query row, [H, hd] heads over keys K/V [L, H, hd] (fp32)."""
    qs = (qrow * scale).bfloat16().float()
    s = torch.einsum("hd,lhd->hl", qs, K)
    if mask is not None:
        s = s.masked_fill(mask[None], float("-inf"))
    p = torch.softmax(s, -1)
    return torch.einsum("hl,lhd->hd", p, V)


@pytest.mark.parametrize("mode", ["self", "self_beam", "cross"])
def test_dec_attn_row(mode):
    C, H, T, S, R, Kb = 256, 8, 16, 37, 6, 3
    hd = C // H
    g = _g(len(mode))
    q = torch.randn(R, C, generator=g).to(DEV).bfloat16()
    x = torch.randn(R, C, generator=g).to(DEV)
    wo = (torch.randn(C, C, generator=g) / 16).to(DEV).bfloat16()
    bo = torch.randn(C, generator=g).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    pos = torch.randn(C, generator=g).to(DEV)
    wq = (torch.randn(C, C, generator=g) / 16).to(DEV).bfloat16()
    bq = torch.randn(C, generator=g).to(DEV)
    xo = torch.empty(R, C, device=DEV)
    q2 = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
    anc, kpm = None, None
    if mode == "cross":
        B = R // Kb
        k = torch.randn(B * S, C, generator=g).to(DEV).bfloat16()
        v = torch.randn(B * S, C, generator=g).to(DEV).bfloat16()
        kpm = torch.zeros(B, S, dtype=torch.uint8)
        kpm[1, -9:] = 1
        kpm = kpm.to(DEV)
        Lk, Lmax, group = S, S, Kb
        rows = [[(r // Kb) * S + j for j in range(S)] for r in range(R)]
        masks = [kpm[r // Kb].bool().cpu() for r in range(R)]
    else:
        k = torch.randn(R * T, C, generator=g).to(DEV).bfloat16()
        v = torch.randn(R * T, C, generator=g).to(DEV).bfloat16()
        Lk, Lmax, group = 11, T, 1
        if mode == "self_beam":
            anc = torch.randint(0, R, (R, T), generator=g, dtype=torch.int32).to(DEV)
            rows = [[int(anc[r, j]) * T + j for j in range(Lk)] for r in range(R)]
        else:
            rows = [[r * T + j for j in range(Lk)] for r in range(R)]
        masks = [None] * R
    call("retr_dec_attn_row", ptr(q), ptr(k), ptr(v), R, C, H, Lk, Lmax, group, ptr(anc),
         ptr(kpm), ptr(x), ptr(wo), ptr(bo), ptr(xo), ptr(gamma), ptr(beta), 1e-12, ptr(pos),
         ptr(wq), ptr(bq), ptr(q2), ops._st())
    scale = 1.0 / math.sqrt(hd)
    kf, vf = k.float().cpu(), v.float().cpu()
    for r in range(R):
        idx = torch.tensor(rows[r])
        o = _attn_ref(q[r].float().cpu().view(H, hd), kf[idx].view(-1, H, hd),
                      vf[idx].view(-1, H, hd), masks[r], scale).reshape(C)
        o = o.bfloat16().float()
        ref_xo = x[r].cpu() + (o @ wo.float().cpu().t() + bo.cpu())
        assert _rel(xo[r], ref_xo) < 1e-4, r
        n = F.layer_norm(ref_xo, (C,), gamma.cpu(), beta.cpu(), 1e-12)
        ref_q2 = (n + pos.cpu()).bfloat16().float() @ wq.float().cpu().t() + bq.cpu()
        assert _rel(q2[r].float(), ref_q2) < 1e-2, r
    # without the second projection: q2 = LN(xo) (bf16)
    call("retr_dec_attn_row", ptr(q), ptr(k), ptr(v), R, C, H, Lk, Lmax, group, ptr(anc),
         ptr(kpm), ptr(x), ptr(wo), ptr(bo), ptr(xo), ptr(gamma), ptr(beta), 1e-12, None, None,
         None, ptr(q2), ops._st())
    ref_n = F.layer_norm(xo, (C,), gamma, beta, 1e-12)
    assert _rel(q2.float(), ref_n) < 1e-2


@pytest.mark.parametrize("R", [7, 64])
def test_dec_ffn_and_reduce(R):
    C, Fh = 256, 2048
    g = _g(R + 1)
    n3 = torch.randn(R, C, generator=g).to(DEV).bfloat16()
    w1 = (torch.randn(Fh, C, generator=g) / 16).to(DEV).bfloat16()
    b1 = torch.randn(Fh, generator=g).to(DEV)
    w2 = (torch.randn(C, Fh, generator=g) / 45).to(DEV).bfloat16()
    b2 = torch.randn(C, generator=g).to(DEV)
    x = torch.randn(R, C, generator=g).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    slabs = torch.empty(Fh // 32, R, C, device=DEV)
    out = torch.empty(R, C, device=DEV)
    n = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
    call("retr_dec_ffn", ptr(n3), R, C, ptr(w1), ptr(b1), ptr(w2), Fh, ptr(slabs), ops._st())
    call("retr_dec_rows", ptr(x), ptr(slabs), Fh // 32, ptr(b2), R, C, ptr(out), ptr(gamma),
         ptr(beta), 1e-12, None, ptr(n), None, ops._st())
    h = torch.relu(n3.float() @ w1.float().t() + b1).bfloat16().float()
    ref = x + (h @ w2.float().t() + b2)
    assert _rel(out, ref) < 1e-4
    assert _rel(n.float(), F.layer_norm(ref, (C,), gamma, beta, 1e-12)) < 1e-2


def test_fused_decode_matches_unfused_cfg5():
    """The fused step (5 launches per layer) against the per-op step on the cfg5 model (bf16):
    first-step logits to bf16 rounding, ids equal up to near-ties (as against the recompute)."""
    from bench import build, cfg5
    from retr_amd.eval_utils.decode import IncrementalGreedy
    from retr_amd.synthetic import synthetic_images
    model, _ = build(cfg5(), DEV)
    model.eval()
    B, T = 8, 128
    img, mask = synthetic_images(B, 224, seed=11, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    fused = IncrementalGreedy(model, fused=True)
    plain = IncrementalGreedy(model, fused=False)
    ids_f = fused(s, T, 101, 102)
    key = next(k for k in model._retr_decode_states if k[0] == "IncrementalGreedy" and k[-1])
    st = model._retr_decode_states[key]
    assert fused._fusable(st) and not plain._fusable(st)
    ids_p = plain(s, T, 101, 102)
    agree = (ids_f == ids_p).float().mean().item()
    assert agree > 0.3, agree           # random weights: near-ties are common (see cfg5 test)
    # first-step logits of both step forms on the same state (cross K/V of this batch)
    with torch.no_grad():
        fused._reset(st, 101)
        fused._step(st, 0, 102)
        lf = st.logits.float().clone()
        fused._reset(st, 101)
        plain._step(st, 0, 102)
        lp = st.logits.float().clone()
    assert _rel(lf, lp) < 2e-2
    # graphs vs eager launches of the fused step: bitwise
    ids_e = IncrementalGreedy(model, use_graphs=False, fused=True)(s, T, 101, 102)
    assert torch.equal(ids_f, ids_e)


@pytest.mark.parametrize("C", [256, 512])
def test_dec_embed_rows_matches_two_launches(C):
    """dec_embed_rows == retr_embed_ln_fwd (one position) followed by retr_dec_rows (LN1 + pos):
    bit-identical x, n and npos."""
    R, V = 70, 1000
    g = _g(C)
    tok = torch.randint(0, V, (R,), generator=g).to(DEV)
    word = torch.randn(V, C, generator=g).to(DEV)
    qp = torch.randn(C, generator=g).to(DEV)
    ge, be = (torch.rand(C, generator=g) + 0.5).to(DEV), torch.randn(C, generator=g).to(DEV)
    g1, b1 = (torch.rand(C, generator=g) + 0.5).to(DEV), torch.randn(C, generator=g).to(DEV)
    x0, x1 = torch.empty(R, C, device=DEV), torch.empty(R, C, device=DEV)
    mean, rstd = torch.empty(R, device=DEV), torch.empty(R, device=DEV)
    n0, p0 = (torch.empty(R, C, dtype=torch.bfloat16, device=DEV) for _ in range(2))
    n1, p1 = (torch.empty(R, C, dtype=torch.bfloat16, device=DEV) for _ in range(2))
    st = ops._st()
    call("retr_embed_ln_fwd", ptr(tok), R, 1, C, ptr(word), ptr(qp), ptr(ge), ptr(be), 1e-12, 0.0,
         0, ptr(x0), ptr(mean), ptr(rstd), st)
    call("retr_dec_rows", ptr(x0), None, 0, None, R, C, None, ptr(g1), ptr(b1), 1e-5, ptr(qp),
         ptr(n0), ptr(p0), st)
    call("retr_dec_embed_rows", ptr(tok), R, C, ptr(word), ptr(qp), ptr(ge), ptr(be), 1e-12,
         ptr(x1), ptr(g1), ptr(b1), 1e-5, ptr(n1), ptr(p1), st)
    assert torch.equal(x0, x1) and torch.equal(n0, n1) and torch.equal(p0, p1)


@pytest.mark.parametrize("B", [3, 64, 100])
def test_greedy_select_matches_argmax_and_update(B):
    """retr_greedy_select == retr_argmax_rows_ws + retr_greedy_update (pred, caption, finished,
    done, tok), including ties (first index wins), rows that hit EOS and the all-finished step."""
    from retr_amd import _lib
    V, Vp, T, eos = 30522, 30528, 16, 102
    g = _g(B)
    logits = torch.randn(B, Vp, generator=g).to(DEV).bfloat16()
    logits[0, 500] = logits[0, 900] = 50.0                     # tie -> 500
    logits[1, eos] = 60.0                                       # finishes
    ws = torch.empty(_lib.load().retr_argmax_workspace(B), dtype=torch.uint8, device=DEV)
    st = ops._st()

    def state():
        cap = torch.zeros(B, T, dtype=torch.long, device=DEV)
        fin = torch.zeros(B, dtype=torch.uint8, device=DEV)
        fin[2 % B] = 1
        done = torch.full((1,), -1, dtype=torch.int32, device=DEV)
        return cap, fin, done, torch.zeros(B, dtype=torch.long, device=DEV), \
            torch.empty(B, dtype=torch.long, device=DEV)

    for step, all_eos in ((3, False), (4, True)):
        if all_eos:
            logits[:, eos] = 70.0
        a, b = state(), state()
        call("retr_argmax_rows_ws", 1, ptr(logits), Vp, B, V, ptr(a[4]), ptr(ws), st)
        call("retr_greedy_update", ptr(a[4]), B, T, step, eos, ptr(a[0]), ptr(a[1]), ptr(a[2]),
             ptr(a[3]), st)
        call("retr_greedy_select", 1, ptr(logits), Vp, B, V, ptr(ws), T, step, eos, ptr(b[4]),
             ptr(b[0]), ptr(b[1]), ptr(b[2]), ptr(b[3]), st)
        for u, v in zip(a, b):
            assert torch.equal(u, v)
        assert int(b[4][0]) == (eos if all_eos else 500)
        assert int(b[2][0]) == (step if all_eos else -1)


@pytest.mark.parametrize("C,H", [(256, 8), (512, 8)])
@pytest.mark.parametrize("beam", [False, True])
def test_dec_heads_self_cross_rows(C, H, beam):
    """One wave per (row, head) (csrc/decode_heads.hip): the self sub-layer (the head's q|k|v
    from LN1(x) (+pos), cache append at position i, attention over keys 0..i with beam ancestry,
    partial out-projection per head), the cross sub-layer (self residual from the head partials,
    LN2 + pos, the head's query, attention over the masked memory with kv_group rows per memory
    row, partial out-projection), and retr_dec_rows' ordered head sum + residual + LN3 --
    against fp32 torch on the same bf16 operands (decode.py:53-81, transformer_modules.py:22-74)."""
    hd = C // H
    R, T, i, S, Kb = 6, 16, 9, 37, (3 if beam else 1)
    g = _g(C + 2 * beam)
    sc = 1.0 / math.sqrt(hd)
    bf = lambda t: t.to(DEV).bfloat16()                       # noqa: E731
    n = bf(torch.randn(R, C, generator=g))
    npos = bf(torch.randn(R, C, generator=g))
    win = bf(torch.randn(3 * C, C, generator=g) / math.sqrt(C))
    bin_ = torch.randn(3 * C, generator=g).to(DEV) * 0.1
    kc = bf(torch.randn(R * T, C, generator=g))
    vc = bf(torch.randn(R * T, C, generator=g))
    kc0, vc0 = kc.clone(), vc.clone()
    anc = torch.randint(0, R, (R, T), generator=g, dtype=torch.int32).to(DEV) if beam else None
    wo = bf(torch.randn(C, C, generator=g) / math.sqrt(C))
    slab = torch.empty(H, R, C, device=DEV)
    call("retr_dec_self_heads", ptr(n), ptr(npos), R, C, H, ptr(win), ptr(bin_), ptr(kc), ptr(vc),
         i, T, ptr(anc), ptr(wo), ptr(slab), ops._st())
    wf = win.float()
    q = (npos.float() @ wf[:C].t() + bin_[:C]).bfloat16().float()
    k = (npos.float() @ wf[C:2 * C].t() + bin_[C:2 * C]).bfloat16().float()
    v = (n.float() @ wf[2 * C:].t() + bin_[2 * C:]).bfloat16().float()
    kv, vv = kc.view(R, T, C), vc.view(R, T, C)
    # the new cache row, and nothing else written
    assert _rel(kv[:, i].float(), k) < 1e-2 and _rel(vv[:, i].float(), v) < 1e-2
    others = torch.ones(T, dtype=torch.bool)
    others[i] = False
    assert torch.equal(kv[:, others], kc0.view(R, T, C)[:, others])
    assert torch.equal(vv[:, others], vc0.view(R, T, C)[:, others])
    kf, vf = kc.float().cpu(), vc.float().cpu()
    for r in range(R):
        rows = [(int(anc[r, j]) if beam else r) * T + j for j in range(i)] + [r * T + i]
        o = _attn_ref(q[r].cpu().view(H, hd), kf[rows].view(-1, H, hd), vf[rows].view(-1, H, hd),
                      None, sc).bfloat16().float()              # [H, hd]
        for h in range(H):
            ref = o[h] @ wo.float().cpu()[:, h * hd:(h + 1) * hd].t()
            assert _rel(slab[h, r], ref) < 1e-2, (r, h)
    # cross sub-layer on those partials
    x = torch.randn(R, C, generator=g).to(DEV)
    bo = torch.randn(C, generator=g).to(DEV) * 0.1
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV) * 0.1
    pos = torch.randn(C, generator=g).to(DEV)
    wq = bf(torch.randn(3 * C, C, generator=g) / math.sqrt(C))
    bq = torch.randn(3 * C, generator=g).to(DEV) * 0.1
    B = R // Kb
    km = bf(torch.randn(B * S, C, generator=g))
    vm = bf(torch.randn(B * S, C, generator=g))
    kpm = torch.zeros(B, S, dtype=torch.uint8)
    kpm[B - 1, -9:] = 1
    kpm = kpm.to(DEV)
    wo2 = bf(torch.randn(C, C, generator=g) / math.sqrt(C))
    xo = torch.empty(R, C, device=DEV)
    slab2 = torch.empty(H, R, C, device=DEV)
    call("retr_dec_cross_heads", ptr(slab), ptr(x), ptr(bo), ptr(xo), R, C, H, ptr(gamma),
         ptr(beta), 1e-5, ptr(pos), ptr(wq), ptr(bq), ptr(km), ptr(vm), S, Kb, ptr(kpm), ptr(wo2),
         ptr(slab2), ops._st())
    ref_xo = x + (slab.sum(0) + bo)
    assert _rel(xo, ref_xo) < 1e-6
    t = (F.layer_norm(ref_xo, (C,), gamma, beta, 1e-5) + pos).bfloat16().float()
    q2 = (t @ wq.float()[:C].t() + bq[:C]).bfloat16().float()
    kmf, vmf = km.float().cpu(), vm.float().cpu()
    for r in range(R):
        b = r // Kb
        idx = torch.arange(b * S, (b + 1) * S)
        o = _attn_ref(q2[r].cpu().view(H, hd), kmf[idx].view(-1, H, hd), vmf[idx].view(-1, H, hd),
                      kpm[b].bool().cpu(), sc).bfloat16().float()
        for h in range(H):
            ref = o[h] @ wo2.float().cpu()[:, h * hd:(h + 1) * hd].t()
            assert _rel(slab2[h, r], ref) < 2e-2, (r, h)
    # the head partials' ordered sum + residual + LN3
    b2 = torch.randn(C, generator=g).to(DEV) * 0.1
    x3 = torch.empty(R, C, device=DEV)
    n3 = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
    call("retr_dec_rows", ptr(xo), ptr(slab2), H, ptr(b2), R, C, ptr(x3), ptr(gamma), ptr(beta),
         1e-5, None, ptr(n3), None, ops._st())
    ref3 = xo + (slab2.sum(0) + b2)
    assert _rel(x3, ref3) < 1e-6
    assert _rel(n3.float(), F.layer_norm(ref3, (C,), gamma, beta, 1e-5)) < 1e-2


def test_dec_heads_step_matches_block_per_row_step():
    """The decode step with the per-(row, head) attention sub-layers (DEC_HEADS) against the
    round-4 block-per-row kernels on the cfg5 model: first-step logits within bf16 rounding
    (only fp32 summation order differs), greedy ids equal up to near-ties, graphs == eager."""
    from bench import build, cfg5
    from retr_amd.eval_utils import decode as dec
    from retr_amd.synthetic import synthetic_images
    model, _ = build(cfg5(), DEV)
    model.eval()
    B, T = 16, 128
    img, mask = synthetic_images(B, 224, seed=12, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    res = {}
    old = dec.DEC_HEADS
    try:
        for heads in (True, False):
            dec.DEC_HEADS = heads
            model._retr_decode_states = {}
            g = dec.IncrementalGreedy(model)
            ids = g(s, T, 101, 102)
            st = next(v for k, v in model._retr_decode_states.items() if k[0] == "IncrementalGreedy")
            with torch.no_grad():
                g._reset(st, 101)
                g._step(st, 0, 102)
                torch.cuda.synchronize()
                res[heads] = (ids, st.logits.float().clone())
            if heads:
                assert st.hslab is not None
                ids_e = dec.IncrementalGreedy(model, use_graphs=False)(s, T, 101, 102)
                assert torch.equal(ids, ids_e)
    finally:
        dec.DEC_HEADS = old
        model._retr_decode_states = {}
    (i1, l1), (i0, l0) = res[True], res[False]
    assert _rel(l1, l0) < 2e-2
    assert (i1 == i0).float().mean().item() > 0.3


@pytest.mark.parametrize("R", [7, 64])
def test_dec_ffn_ln_matches_rows_then_ffn(R):
    """retr_dec_ffn_ln (the FFN input LayerNorm of the head partials in the FFN prologue) against
    retr_dec_rows (ordered head-partial sum + residual + LN) followed by retr_dec_ffn: the
    residual bitwise equal, the FFN partial slabs within bf16 rounding of the LN output."""
    C, Fh, H = 256, 2048, 8
    g = _g(R + 7)
    x = torch.randn(R, C, generator=g).to(DEV)
    hs = torch.randn(H, R, C, generator=g).to(DEV)
    bo = torch.randn(C, generator=g).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    w1 = (torch.randn(Fh, C, generator=g) / 16).to(DEV).bfloat16()
    b1 = torch.randn(Fh, generator=g).to(DEV)
    w2 = (torch.randn(C, Fh, generator=g) / 45).to(DEV).bfloat16()
    xo0, xo1 = torch.empty(R, C, device=DEV), torch.empty(R, C, device=DEV)
    n3 = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
    s0 = torch.empty(Fh // 32, R, C, device=DEV)
    s1 = torch.empty_like(s0)
    st = ops._st()
    call("retr_dec_rows", ptr(x), ptr(hs), H, ptr(bo), R, C, ptr(xo0), ptr(gamma), ptr(beta),
         1e-5, None, ptr(n3), None, st)
    call("retr_dec_ffn", ptr(n3), R, C, ptr(w1), ptr(b1), ptr(w2), Fh, ptr(s0), st)
    call("retr_dec_ffn_ln", ptr(x), ptr(hs), H, ptr(bo), ptr(gamma), ptr(beta), 1e-5, ptr(xo1), R,
         C, ptr(w1), ptr(b1), ptr(w2), Fh, ptr(s1), st)
    assert torch.equal(xo0, xo1)
    assert _rel(s1, s0) < 1e-2


def test_dec_self_heads_ln_matches_rows_then_heads():
    """retr_dec_self_heads_ln (the previous layer's FFN partials + residual + LN1 (+qpos) in the
    self-attention prologue) against retr_dec_rows followed by retr_dec_self_heads: the
    residual, the cache row and the head partials within fp32 reassociation / bf16 rounding."""
    C, H, R, T, i, ns = 256, 8, 64, 16, 5, 32
    g = _g(99)
    bf = lambda t: t.to(DEV).bfloat16()                       # noqa: E731
    x = torch.randn(R, C, generator=g).to(DEV)
    slabs = torch.randn(ns, R, C, generator=g).to(DEV) * 0.1
    b2 = torch.randn(C, generator=g).to(DEV) * 0.1
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV) * 0.1
    qp = torch.randn(C, generator=g).to(DEV)
    win = bf(torch.randn(3 * C, C, generator=g) / math.sqrt(C))
    bin_ = torch.randn(3 * C, generator=g).to(DEV) * 0.1
    wo = bf(torch.randn(C, C, generator=g) / math.sqrt(C))
    kc0 = bf(torch.randn(R * T, C, generator=g))
    vc0 = bf(torch.randn(R * T, C, generator=g))
    st = ops._st()
    # reference: rows then heads
    x1 = torch.empty(R, C, device=DEV)
    n = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
    npos = torch.empty_like(n)
    call("retr_dec_rows", ptr(x), ptr(slabs), ns, ptr(b2), R, C, ptr(x1), ptr(gamma), ptr(beta),
         1e-5, ptr(qp), ptr(n), ptr(npos), st)
    kc1, vc1 = kc0.clone(), vc0.clone()
    s1 = torch.empty(H, R, C, device=DEV)
    call("retr_dec_self_heads", ptr(n), ptr(npos), R, C, H, ptr(win), ptr(bin_), ptr(kc1),
         ptr(vc1), i, T, None, ptr(wo), ptr(s1), st)
    # fused prologue
    x2 = torch.empty(R, C, device=DEV)
    kc2, vc2 = kc0.clone(), vc0.clone()
    s2 = torch.empty(H, R, C, device=DEV)
    call("retr_dec_self_heads_ln", None, None, R, C, H, ptr(win), ptr(bin_), ptr(kc2), ptr(vc2), i,
         T, None, ptr(wo), ptr(s2), ptr(x), ptr(slabs), ns, ptr(b2), ptr(gamma), ptr(beta), 1e-5,
         ptr(qp), ptr(x2), st)
    assert _rel(x2, x1) < 1e-6
    assert _rel(kc2.float(), kc1.float()) < 1e-2 and _rel(vc2.float(), vc1.float()) < 1e-2
    assert _rel(s2, s1) < 2e-2


@pytest.mark.parametrize("fold", [False, True])
def test_dec_fold_rows_step_matches(fold):
    """The three-launch decoder layer (DEC_FOLD_ROWS: FFN residual + next LN1 in the self prologue,
    cross residual + LN3 in the FFN prologue, 64 hidden units per FFN block) against the
    five-launch one on the cfg5 model: first-step logits within bf16 rounding, graphs == eager."""
    from bench import build, cfg5
    from retr_amd.eval_utils import decode as dec
    from retr_amd.synthetic import synthetic_images
    model, _ = build(cfg5(), DEV)
    model.eval()
    B, T = 16, 128
    img, mask = synthetic_images(B, 224, seed=13, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    old = (dec.DEC_HEADS, dec.DEC_FFN_LN, dec.DEC_FOLD_ROWS)
    res = []
    try:
        for f in (fold, False):
            dec.DEC_HEADS, dec.DEC_FFN_LN, dec.DEC_FOLD_ROWS = True, True, f
            model._retr_decode_states = {}
            gr = dec.IncrementalGreedy(model)
            ids = gr(s, T, 101, 102)
            st = next(v for k, v in model._retr_decode_states.items() if k[0] == "IncrementalGreedy")
            with torch.no_grad():
                gr._reset(st, 101)
                gr._step(st, 0, 102)
                torch.cuda.synchronize()
                res.append(st.logits.float().clone())
            if f:
                ids_e = dec.IncrementalGreedy(model, use_graphs=False)(s, T, 101, 102)
                assert torch.equal(ids, ids_e)
    finally:
        dec.DEC_HEADS, dec.DEC_FFN_LN, dec.DEC_FOLD_ROWS = old
        model._retr_decode_states = {}
    assert _rel(res[0], res[1]) < 2e-2


@pytest.mark.parametrize("rb,kv_group,prologue", [(5, 5, False), (5, 5, True), (2, 1, False),
                                                  (4, 2, True), (4, 8, False)])
def test_dec_heads_multi_row_matches_per_row(rb, kv_group, prologue):
    """retr_dec_self_heads_mr / retr_dec_cross_heads_mr (rb rows x one head per block, weight
    slices -- and memory keys / values when kv_group % rb == 0 -- staged in LDS) against the
    per-(row, head) kernels on the same operands: identical arithmetic, so every output (head
    partials, cache rows, residual) is bit-identical; beam ancestry, masked memory keys."""
    C, H = 256, 8
    R, T, i, S = 40, 32, 21, 197
    g = _g(rb * 10 + kv_group + prologue)
    bf = lambda t: t.to(DEV).bfloat16()                       # noqa: E731
    n = bf(torch.randn(R, C, generator=g))
    npos = bf(torch.randn(R, C, generator=g))
    win = bf(torch.randn(3 * C, C, generator=g) / math.sqrt(C))
    bin_ = torch.randn(3 * C, generator=g).to(DEV) * 0.1
    kc = bf(torch.randn(R * T, C, generator=g))
    vc = bf(torch.randn(R * T, C, generator=g))
    anc = torch.randint(0, R, (R, T), generator=g, dtype=torch.int32).to(DEV)
    wo = bf(torch.randn(C, C, generator=g) / math.sqrt(C))
    nsl = 4
    xin = torch.randn(R, C, generator=g).to(DEV)
    slabs = torch.randn(nsl, R, C, generator=g).to(DEV) * 0.3
    b2 = torch.randn(C, generator=g).to(DEV) * 0.1
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV) * 0.1
    qpos = torch.randn(C, generator=g).to(DEV)
    outs = []
    _lib.load().retr_tune(31, 1)          # the per-row kernels' two-wave layout (the mr layout)
    for r_b in (1, rb):
        kc1, vc1 = kc.clone(), vc.clone()
        slab = torch.full((H, R, C), float("nan"), device=DEV)
        xout = torch.full((R, C), float("nan"), device=DEV)
        if prologue:
            call("retr_dec_self_heads_mr", None, None, R, C, H, ptr(win), ptr(bin_), ptr(kc1),
                 ptr(vc1), i, T, ptr(anc), ptr(wo), ptr(slab), ptr(xin), ptr(slabs), nsl, ptr(b2),
                 ptr(gamma), ptr(beta), 1e-5, ptr(qpos), ptr(xout), r_b, ops._st())
        else:
            call("retr_dec_self_heads_mr", ptr(n), ptr(npos), R, C, H, ptr(win), ptr(bin_),
                 ptr(kc1), ptr(vc1), i, T, ptr(anc), ptr(wo), ptr(slab), None, None, 0, None,
                 None, None, 0.0, None, None, r_b, ops._st())
        B = R // kv_group
        km = bf(torch.randn(B * S, C, generator=_g(7)))
        vm = bf(torch.randn(B * S, C, generator=_g(8)))
        kpm = torch.zeros(B, S, dtype=torch.uint8)
        kpm[B - 1, -13:] = 1
        kpm = kpm.to(DEV)
        x = torch.randn(R, C, generator=_g(9)).to(DEV)
        wq = bf(torch.randn(3 * C, C, generator=_g(10)) / math.sqrt(C))
        bq = torch.randn(3 * C, generator=_g(11)).to(DEV) * 0.1
        wo2 = bf(torch.randn(C, C, generator=_g(12)) / math.sqrt(C))
        xo = torch.full((R, C), float("nan"), device=DEV)
        slab2 = torch.full((H, R, C), float("nan"), device=DEV)
        call("retr_dec_cross_heads_mr", ptr(slab), ptr(x), ptr(b2), ptr(xo), R, C, H, ptr(gamma),
             ptr(beta), 1e-5, ptr(qpos), ptr(wq), ptr(bq), ptr(km), ptr(vm), S, kv_group,
             ptr(kpm), ptr(wo2), ptr(slab2), r_b, ops._st())
        torch.cuda.synchronize()
        outs.append((slab, kc1, vc1, xo, slab2) + ((xout,) if prologue else ()))
    _lib.load().retr_tune(31, 0)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert not torch.isnan(outs[1][-1]).any()


def test_dec_multi_row_beam_step_matches():
    """Beam 5 decode with the multi-row attention blocks (the automatic choice: a block per beam
    group x head) against a block per (row, head) on the cfg5 model: identical captions and
    first-step logits (bit-identical kernels), graphs == eager."""
    from bench import build, cfg5
    from retr_amd.eval_utils import decode as dec
    from retr_amd.synthetic import synthetic_images
    model, _ = build(cfg5(), DEV)
    model.eval()
    B, T = 8, 128
    img, mask = synthetic_images(B, 224, seed=17, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    old = dec.DEC_ROWS_PER_BLOCK, dec.DEC_EMBED_FOLD
    res = []
    try:
        for rb in (None, 1):
            # (the embedding fold runs on per-row blocks only: off for both, same arithmetic)
            dec.DEC_ROWS_PER_BLOCK, dec.DEC_EMBED_FOLD = rb, False
            _lib.load().retr_tune(31, 1)    # two-wave per-row kernels: the mr kernels' arithmetic
            model._retr_decode_states = {}
            bm = dec.IncrementalBeam(model, 5)
            ids = bm(s, T, 101, 102)
            res.append(ids)
            if rb is None:
                assert dec._rows_per_block(B * 5, 256, 8, 5, 1, 197) == (5, 5)
                ids_e = dec.IncrementalBeam(model, 5, use_graphs=False)(s, T, 101, 102)
                assert torch.equal(ids, ids_e)
    finally:
        dec.DEC_ROWS_PER_BLOCK, dec.DEC_EMBED_FOLD = old
        _lib.load().retr_tune(31, 0)
        model._retr_decode_states = {}
    assert torch.equal(res[0], res[1])


def test_dec_self_heads_embed_matches_embed_rows_then_heads():
    """retr_dec_self_heads_embed (DecoderEmbeddings + LN1 in the first self-attention launch)
    against retr_dec_embed_rows + retr_dec_self_heads on the same operands: residual x within
    fp32 reassociation of the LayerNorm sums, head partials and cache rows within bf16 rounding."""
    C, H, R, T, i, V = 256, 8, 16, 32, 11, 500
    g = _g(77)
    bf = lambda t: t.to(DEV).bfloat16()                       # noqa: E731
    tok = torch.randint(0, V, (R,), generator=g).to(DEV)
    word = torch.randn(V, C, generator=g).to(DEV)
    qp = torch.randn(C, generator=g).to(DEV)
    ge, g1 = [(torch.rand(C, generator=g) + 0.5).to(DEV) for _ in range(2)]
    be, b1 = [(torch.randn(C, generator=g) * 0.1).to(DEV) for _ in range(2)]
    win = bf(torch.randn(3 * C, C, generator=g) / math.sqrt(C))
    bin_ = torch.randn(3 * C, generator=g).to(DEV) * 0.1
    kc = bf(torch.randn(R * T, C, generator=g))
    vc = bf(torch.randn(R * T, C, generator=g))
    wo = bf(torch.randn(C, C, generator=g) / math.sqrt(C))
    outs = []
    for fused in (True, False):
        k1, v1 = kc.clone(), vc.clone()
        x = torch.full((R, C), float("nan"), device=DEV)
        slab = torch.full((H, R, C), float("nan"), device=DEV)
        if fused:
            call("retr_dec_self_heads_embed", ptr(tok), ptr(word), ptr(ge), ptr(be), 1e-12, R, C,
                 H, ptr(win), ptr(bin_), ptr(k1), ptr(v1), i, T, None, ptr(wo), ptr(slab),
                 ptr(g1), ptr(b1), 1e-5, ptr(qp), ptr(x), ops._st())
        else:
            n = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
            npos = torch.empty_like(n)
            call("retr_dec_embed_rows", ptr(tok), R, C, ptr(word), ptr(qp), ptr(ge), ptr(be),
                 1e-12, ptr(x), ptr(g1), ptr(b1), 1e-5, ptr(n), ptr(npos), ops._st())
            call("retr_dec_self_heads", ptr(n), ptr(npos), R, C, H, ptr(win), ptr(bin_),
                 ptr(k1), ptr(v1), i, T, None, ptr(wo), ptr(slab), ops._st())
        torch.cuda.synchronize()
        outs.append((x, slab, k1, v1))
    (x1, s1, k1, v1), (x0, s0, k0, v0) = outs
    ref = F.layer_norm(word[tok] + qp, (C,), ge, be, 1e-12)
    assert _rel(x0, ref) < 1e-5 and _rel(x1, ref) < 1e-5
    assert _rel(s1, s0) < 2e-2
    assert _rel(k1.float(), k0.float()) < 1e-2 and _rel(v1.float(), v0.float()) < 1e-2


@pytest.mark.parametrize("embed", [True, False])
def test_dec_embed_fold_step_matches(embed):
    """The decode step with the embeddings folded into the first self-attention launch
    (DEC_EMBED_FOLD) against the separate embed launch on the cfg5 model: first-step logits
    within bf16 rounding, graphs == eager."""
    from bench import build, cfg5
    from retr_amd.eval_utils import decode as dec
    from retr_amd.synthetic import synthetic_images
    model, _ = build(cfg5(), DEV)
    model.eval()
    B, T = 16, 128
    img, mask = synthetic_images(B, 224, seed=21, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    old = dec.DEC_EMBED_FOLD
    res = []
    try:
        for f in (embed, False):
            dec.DEC_EMBED_FOLD = f
            model._retr_decode_states = {}
            gr = dec.IncrementalGreedy(model)
            ids = gr(s, T, 101, 102)
            st = next(v for k, v in model._retr_decode_states.items() if k[0] == "IncrementalGreedy")
            with torch.no_grad():
                gr._reset(st, 101)
                gr._step(st, 0, 102)
                torch.cuda.synchronize()
                res.append(st.logits.float().clone())
            if f:
                ids_e = dec.IncrementalGreedy(model, use_graphs=False)(s, T, 101, 102)
                assert torch.equal(ids, ids_e)
    finally:
        dec.DEC_EMBED_FOLD = old
        model._retr_decode_states = {}
    assert _rel(res[0], res[1]) < 2e-2


@pytest.mark.parametrize("R", [5, 320])
def test_dec_ffn_ln_hidden_block_widths_agree(R):
    """retr_dec_ffn_ln64 / retr_dec_ffn_ln128 (64 / 128 hidden units per block) against
    retr_dec_rows + retr_dec_ffn: the residual bitwise equal, the sum of each variant's partial
    slabs (the FFN output before its bias) within bf16 rounding of the LN output."""
    C, Fh, H = 256, 2048, 8
    g = _g(R + 11)
    x = torch.randn(R, C, generator=g).to(DEV)
    hs = torch.randn(H, R, C, generator=g).to(DEV)
    bo = torch.randn(C, generator=g).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    w1 = (torch.randn(Fh, C, generator=g) / 16).to(DEV).bfloat16()
    b1 = torch.randn(Fh, generator=g).to(DEV)
    w2 = (torch.randn(C, Fh, generator=g) / 45).to(DEV).bfloat16()
    st = ops._st()
    xo0 = torch.empty(R, C, device=DEV)
    n3 = torch.empty(R, C, dtype=torch.bfloat16, device=DEV)
    s0 = torch.empty(Fh // 32, R, C, device=DEV)
    call("retr_dec_rows", ptr(x), ptr(hs), H, ptr(bo), R, C, ptr(xo0), ptr(gamma), ptr(beta),
         1e-5, None, ptr(n3), None, st)
    call("retr_dec_ffn", ptr(n3), R, C, ptr(w1), ptr(b1), ptr(w2), Fh, ptr(s0), st)
    ref = s0.sum(0)
    for name, hb in (("retr_dec_ffn_ln64", 64), ("retr_dec_ffn_ln128", 128)):
        xo = torch.full((R, C), float("nan"), device=DEV)
        sl = torch.full((Fh // hb, R, C), float("nan"), device=DEV)
        call(name, ptr(x), ptr(hs), H, ptr(bo), ptr(gamma), ptr(beta), 1e-5, ptr(xo), R, C,
             ptr(w1), ptr(b1), ptr(w2), Fh, ptr(sl), st)
        torch.cuda.synchronize()
        assert torch.equal(xo, xo0), name
        assert _rel(sl.sum(0), ref) < 1e-2, name


@pytest.mark.parametrize("M,N,K,relu,res", [(64, 256, 256, 0, True), (37, 2048, 256, 1, False),
                                            (64, 256, 2048, 0, True), (2, 30528, 512, 0, False),
                                            (16, 512, 512, 1, False)])
def test_dec_linear_f32_matches_torch(M, N, K, relu, res):
    """retr_dec_linear_f32 (the fp32 parity-mode decode linears) against fp32 torch: within fp32
    reassociation; strided output rows (the cache append) and the residual."""
    g = _g(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    r = torch.randn(M, N, generator=g).to(DEV) if res else None
    big = torch.full((M, 2 * N), float("nan"), device=DEV)
    y = big[:, 3:3 + N] if N % 4 else big[:, N:]
    call("retr_dec_linear_f32", ptr(x), K, ptr(w), K, ptr(b), ptr(y), y.stride(0), M, N, K, relu,
         ptr(r), N if res else 0, ops._st())
    torch.cuda.synchronize()
    ref = x.double() @ w.double().t() + b.double()
    if relu:
        ref = ref.clamp_min(0)
    if res:
        ref = ref + r.double()
    assert _rel(y, ref) < 1e-6


def test_fused_decode_head_dim64_long_memory_takes_block_per_row_step():
    """Head dim 64 with 289 memory keys (> 256, the per-(row, head) kernels' limit at that head
    dim): the fused greedy step must route to the block-per-row kernels (up to 512 keys) instead
    of failing partway through decoding, and agree with the per-op step (bf16 rounding)."""
    from tests.helpers import make_config
    from retr_amd.eval_utils import decode as dec
    from retr_amd.models.caption import build_model
    from retr_amd.synthetic import synthetic_images, synthetic_state_dict
    cfg = make_config(backbone="ResNet18", hidden=256, layers=(1, 2), vocab=1000, max_pos=16,
                      nheads=4, ffn=512, dtype="bf16")
    model, _ = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=5))
    model.to(DEV).eval()
    B, T = 4, 16
    img, mask = synthetic_images(B, 544, seed=13, pad_band=True)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    fused = dec.IncrementalGreedy(model, fused=True)
    ids_f = fused(s, T, 101, 102)
    st = next(v for k, v in model._retr_decode_states.items() if k[0] == "IncrementalGreedy" and k[-1])
    assert st.S == 289 and fused._fusable(st) and not fused._heads_ok(st)
    assert st.hslab is None                       # the per-(row, head) kernels never ran
    plain = dec.IncrementalGreedy(model, fused=False)
    ids_p = plain(s, T, 101, 102)
    assert (ids_f == ids_p).float().mean().item() > 0.3
    with torch.no_grad():
        fused._reset(st, 101)
        fused._step(st, 0, 102)
        lf = st.logits.float().clone()
        fused._reset(st, 101)
        plain._step(st, 0, 102)
        lp = st.logits.float().clone()
    assert _rel(lf, lp) < 2e-2
