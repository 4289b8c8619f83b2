"""Whole-path parity on the GPU: retr_amd (HIP kernels, fp32 parity mode) vs the CPU oracle.

Bars (BASELINE.json north_star): logits/loss within 1e-3 (fp32), token ids bit-exact under
greedy decode.  The oracle is the CPU restatement pinned to the reference by
tests/golden/*.npz (tests/test_oracle.py).
"""
import pytest
import torch

from oracle import model as orc
from retr_amd.eval_utils.decode import (IncrementalGreedy, greedy,
                                        greedy_reference_algorithm)
from retr_amd.models.caption import build_model
from retr_amd.models.utils import NestedTensor
from retr_amd.synthetic import synthetic_captions, synthetic_images, synthetic_state_dict
from tests.helpers import PARITY_CASES, make_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(case, dtype="fp32", seed=42):
    kw, size, B = PARITY_CASES[case]
    cfg = make_config(dtype=dtype, **kw)
    model, crit = build_model(cfg)
    sd = synthetic_state_dict(model, seed=seed)
    model.load_state_dict(sd)
    model.to(DEV)
    images, mask = synthetic_images(B, size, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=2)
    return cfg, model, crit, sd, images, mask, caps, cap_mask


def _max_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("case", ["micro_r18", "micro_r50_dil", "cfg1"])
def test_forward_backward_matches_oracle(case):
    cfg, model, crit, sd, images, mask, caps, cap_mask = _setup(case)
    model.train()
    out = model(NestedTensor(images.to(DEV), mask.to(DEV)), caps[:, :-1].to(DEV),
                cap_mask[:, :-1].to(DEV))
    loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
    loss.backward()

    trainable = {n for n, p in model.named_parameters() if p.requires_grad}
    sdo = {k: (v.clone().requires_grad_(True) if k in trainable else v) for k, v in sd.items()}
    lo = orc.caption_forward(sdo, cfg, images, mask, caps[:, :-1], cap_mask[:, :-1])
    loss_o = orc.caption_loss(lo, caps[:, 1:])
    loss_o.backward()

    assert out.shape == lo.shape
    assert _max_rel(out, lo) < 1e-3, case
    assert abs(loss.item() - loss_o.item()) <= 1e-3 * abs(loss_o.item())
    worst = 0.0
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        g, go = p.grad, sdo[n].grad
        assert g is not None and go is not None, n
        denom = go.norm().item()
        if denom == 0:
            continue
        e = ((g.double().cpu() - go.double()).norm() / denom).item()
        worst = max(worst, e)
        assert e < 2e-3, (n, e)


@pytest.mark.parametrize("case", ["micro_r18", "micro_r50_dil"])
def test_attention_maps_match_oracle(case):
    cfg, model, crit, sd, images, mask, caps, cap_mask = _setup(case)
    model.eval()
    with torch.no_grad():
        out, att = model(NestedTensor(images.to(DEV), mask.to(DEV)), caps[:, :-1].to(DEV),
                         cap_mask[:, :-1].to(DEV), return_attention=True)
    lo, atto = orc.caption_forward(sd, cfg, images, mask, caps[:, :-1], cap_mask[:, :-1],
                                   return_attention=True)
    assert set(att) == set(atto)
    for k in att:
        assert att[k].shape == atto[k].shape, k
        assert _max_rel(att[k], atto[k]) < 1e-3, k


def _oracle_greedy(cfg, sd, images, mask, eos):
    def fwd(c, m):
        return orc.caption_forward(sd, cfg, images, mask, c, m)
    with torch.no_grad():
        return orc.greedy(fwd, images.shape[0], cfg.max_position_embeddings, 101, eos)


@pytest.mark.parametrize("case", ["micro_r18", "micro_r50_dil"])
def test_greedy_ids_bit_exact(case):
    cfg, model, crit, sd, images, mask, caps, cap_mask = _setup(case)
    model.eval()
    T = cfg.max_position_embeddings
    samples = [NestedTensor(images.to(DEV), mask.to(DEV))]
    ids_never = _oracle_greedy(cfg, sd, images, mask, eos=-1)
    # EOS choices: never emitted / emitted by row 0 mid-sequence (early finish of one row) /
    # the token row 0 emits at step 1 for every row that also emits it (full early return)
    for eos in (-1, int(ids_never[0, 6]), int(ids_never[0, 1])):
        ids = greedy(samples, model, max_len=T, bos_token=101, eos_token=eos)   # hipGraphs
        ids_eager = IncrementalGreedy(model, use_graphs=False)(samples[0], T, 101, eos)
        assert torch.equal(ids, ids_eager), (case, eos)       # graph replay == eager launches
        ids_full = greedy_reference_algorithm(samples, model, T, 101, eos)
        assert torch.equal(ids, ids_full), (case, eos)        # KV cache == full recompute ids
        ids_o = _oracle_greedy(cfg, sd, images, mask, eos)
        assert torch.equal(ids.cpu(), ids_o), (case, eos)      # == reference algorithm on CPU


def test_bf16_training_step_runs():
    cfg, model, crit, sd, images, mask, caps, cap_mask = _setup("micro_r50_dil", dtype="bf16")
    cfg.dropout = 0.1
    model.train()
    opt = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    losses = []
    for _ in range(3):
        out = model(NestedTensor(images.to(DEV), mask.to(DEV)), caps[:, :-1].to(DEV),
                    cap_mask[:, :-1].to(DEV))
        loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.1)
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("case", list(PARITY_CASES))
def test_hip_path_matches_reference_goldens(case):
    """Directly against the vectors the reference produced (tests/golden/*.npz)."""
    import os
    import numpy as np
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             f"{case}.npz"))
    cfg, model, crit, sd, images, mask, caps, cap_mask = _setup(case)
    model.train()
    out = model(NestedTensor(images.to(DEV), mask.to(DEV)), caps[:, :-1].to(DEV),
                cap_mask[:, :-1].to(DEV))
    loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
    loss.backward()
    lg = out.detach().float().cpu()
    ref = torch.from_numpy(g["logits"]) if "logits" in g else torch.from_numpy(g["logits_at"])
    if "logits" not in g:
        lg = lg[:, list(g["positions"])]
    assert ((lg - ref).abs().max() / ref.abs().max()).item() < 1e-3
    assert abs(loss.item() - float(g["loss"])) <= 1e-3 * abs(float(g["loss"]))
    names = list(g["grad_names"])
    norms = np.array([dict(model.named_parameters())[n].grad.norm().item() for n in names])
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=2e-3)
    if "greedy_eos" in g:
        model.eval()
        samples = [NestedTensor(images.to(DEV), mask.to(DEV))]
        for i, eos in enumerate(g["greedy_eos"]):
            ids = greedy(samples, model, max_len=cfg.max_position_embeddings, bos_token=101,
                         eos_token=int(eos))
            np.testing.assert_array_equal(ids.cpu().numpy(), g[f"greedy/eos{i}"])


def test_cat_tail_matches_unfused():
    """bf16 backbone with the fused bottleneck tail (retr_conv1x1_fwd_cat on the first block of
    every layer: stride-1 downsample in layer1 and dilated layer4, stride 2 in layer2/3) vs the unfused downsample + residual path: logits and loss within bf16
    tolerance of each other, and every gradient no further from the fp32 model's than the
    unfused path's is (the fused path skips one bf16 rounding of the downsample output; in a
    micro bf16 backbone either rounding moves deep weight gradients by a few percent)."""
    _, m32, crit32, _, images, mask, caps, cap_mask = _setup("micro_r50_dil", dtype="fp32")
    cfg, model, crit, sd, *_ = _setup("micro_r50_dil", dtype="bf16")
    bb = next(m for m in model.modules() if hasattr(m, "runner") and hasattr(m, "body"))
    runner = bb.runner(torch.bfloat16)
    runner.use_fused = False          # this test is about the fused tail of the unfused blocks
    samples = NestedTensor(images.to(DEV), mask.to(DEV))

    def run(mdl, cr):
        mdl.zero_grad(set_to_none=True)
        out = mdl(samples, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
        loss = cr(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
        loss.backward()
        return (out.detach().float().clone(), loss.item(),
                {n: p.grad.detach().double().clone() for n, p in mdl.named_parameters()
                 if p.grad is not None})

    o32, l32, g32 = run(m32, crit32)
    runner.use_cat = True
    o1, l1, g1 = run(model, crit)
    assert runner.cat_used == ["layer1.0", "layer2.0", "layer3.0", "layer4.0"], runner.cat_used
    runner.use_cat = False
    o0, l0, g0 = run(model, crit)
    runner.use_cat = True
    assert _max_rel(o1, o0) < 2e-2
    assert abs(l1 - l0) < 1e-2 * abs(l0)
    assert g1.keys() == g0.keys() == g32.keys() and len(g1) > 0

    def err(g, n):
        return ((g[n] - g32[n]).norm() / (g32[n].norm() + 1e-30)).item()

    e1 = sum(err(g1, n) for n in g1) / len(g1)
    e0 = sum(err(g0, n) for n in g0) / len(g0)
    assert e1 <= 1.25 * e0 + 1e-3, (e1, e0)
    for n in g1:
        assert err(g1, n) <= 2.0 * err(g0, n) + 2e-2, (n, err(g1, n), err(g0, n))


def test_fused_layer1_bottlenecks_bitwise_in_model():
    """The cfg2-shaped bf16 model (ResNet-50, 640x640, batch 2): the frozen layer1 blocks run as
    retr_bottleneck_s1_fwd launches, and the training forward's logits and loss are bitwise
    those of the unfused block path (three conv launches, or two + the fused tail)."""
    from bench import build, cfg2
    cfg = cfg2()
    cfg.dropout = 0.0
    model, crit = build(cfg, DEV)
    model.train()
    bb = next(m for m in model.modules() if hasattr(m, "runner") and hasattr(m, "body"))
    runner = bb.runner(torch.bfloat16)
    img, mask = synthetic_images(2, 640, seed=21)
    caps, cm = synthetic_captions(2, cfg.max_position_embeddings, cfg.vocab_size, seed=22)
    s = NestedTensor(img.to(DEV), mask.to(DEV))
    outs = []
    for fused in (True, False):
        runner.use_fused = fused
        with torch.no_grad():
            out = model(s, caps[:, :-1].to(DEV), cm[:, :-1].to(DEV))
            loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV)).item()
        outs.append((out.float().clone(), loss))
        expect = ["layer1.0", "layer1.1", "layer1.2"] if fused else []
        assert runner.fused_used == expect, runner.fused_used
    runner.use_fused = True
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]


@pytest.mark.parametrize("hidden", [64, 256])
def test_fused_ln_dropout_backward_matches_unfused(hidden):
    """bf16 transformer blocks: the fused backward (each block's LayerNorm backward also writes
    the previous block's bf16 dropout(dx), and leaves its dgamma/dbeta partial rows to the
    weight-gradient slab-sum launch) against the unfused launches, residual dropout on.  Every
    gradient is bitwise equal except the LayerNorm parameters (partials added in another fixed
    order, rel 1e-5); the memory gradients of the six cross-attention blocks are summed in the
    data-gradient GEMM epilogues instead of by autograd (bf16 tolerance upstream of the memory);
    hidden 256 runs the 4-wide kernel with the in-kernel dropout copy, hidden 64 the generic
    kernel + retr_dropout_apply inside retr_layernorm_bwd2."""
    from retr_amd import ops
    cfg = make_config(backbone="ResNet18", hidden=hidden, layers=(2, 2), vocab=1000, max_pos=16,
                      ffn=2 * hidden, dtype="bf16", dropout=0.1)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=3))
    model.to(DEV).train()
    images, mask = synthetic_images(2, 64, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(2, 16, 1000, seed=2)
    s = NestedTensor(images.to(DEV), mask.to(DEV))
    ctr = ops._seed_state["ctr"]
    res = []
    try:
        for fuse in (True, False):
            ops.FUSE_LN_BWD = fuse
            ops._seed_state["ctr"] = ctr
            ops.DBR_STATS.update(hit=0, miss=0)
            model.zero_grad(set_to_none=True)
            out = model(s, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
            loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
            loss.backward()
            torch.cuda.synchronize()
            res.append(({n: p.grad.detach().clone() for n, p in model.named_parameters()
                         if p.grad is not None}, dict(ops.DBR_STATS), loss.item()))
    finally:
        ops.FUSE_LN_BWD = True
    (g1, st1, l1), (g0, st0, l0) = res
    assert l1 == l0
    # every block but the first of each stack takes its incoming gradient from the cache
    assert st1["hit"] == (2 * 2 - 1) + (3 * 2 - 1), st1
    assert st0["hit"] == 0
    assert g1.keys() == g0.keys() and len(g1) > 0
    def rel(n):
        return ((g1[n] - g0[n]).double().norm() / (g0[n].double().norm() + 1e-30)).item()

    for n in g1:
        dec = "transformer.decoder" in n or n.startswith("mlp") or "embeddings" in n
        if dec and (".norm" in n or "position_embeddings" in n):
            # partials / per-block contributions added in another fixed order
            assert rel(n) < 1e-5, (n, rel(n))
        elif dec:
            assert torch.equal(g1[n], g0[n]), n
        else:
            # upstream of the memory: the six cross-attention blocks' bf16 memory gradients
            # are summed in the GEMM epilogues (one bf16 rounding fewer per add)
            assert rel(n) < 2e-2, (n, rel(n))


@pytest.mark.parametrize("extra_use", [False, True])
def test_shared_memory_gradient_is_sum_of_block_contributions(extra_use):
    """The bf16 decoder sums the six cross-attention blocks' memory gradients (dmem, dmem_pos)
    in ONE shared buffer inside the data-gradient GEMM epilogues (ops._shared_grad: the first
    contributor writes it, later ones add the running sum as the epilogue addend, the last
    returns it).  Checked directly against the fp32 sum of the per-block contributions that
    the unfused path returns one by one: every element within a few bf16 roundings of the sum,
    the norm within 1e-2 -- a dropped, doubled or misplaced contributor is off by ~1/6 of the
    sum.  ``extra_use``: the memory also feeds a plain autograd op, so autograd accumulates
    the shared buffer with a foreign gradient."""
    from retr_amd import ops
    cfg = make_config(backbone="ResNet18", hidden=64, layers=(1, 6), vocab=1000, max_pos=16,
                      ffn=128, dtype="bf16", dropout=0.0)
    model, _ = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=5))
    model.to(DEV).train()
    tr = model.transformer
    B, S, T, C = 2, 24, 16, 64
    g = torch.Generator().manual_seed(7)
    mem0 = torch.randn(B * S, C, generator=g)
    memp0 = mem0 + 0.1 * torch.randn(B * S, C, generator=g)
    mem0, memp0 = mem0.to(DEV, torch.bfloat16), memp0.to(DEV, torch.bfloat16)
    kpm = torch.zeros(B, S, dtype=torch.uint8, device=DEV)
    kpm[1, S - 5:] = 1
    caps, cap_mask = synthetic_captions(B, T, 1000, seed=3)
    tgt, tm = caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV)
    w_hs = torch.randn(B * T, C, generator=g).to(DEV)
    w_x = torch.randn(B * S, C, generator=g).to(DEV)
    contrib = []
    orig = ops._CrossAttnBlock.backward

    def recording(ctx, *grads):
        r = orig(ctx, *grads)
        contrib.append((r[6].float().clone(), r[7].float().clone()))
        return r

    res = {}
    try:
        for fuse in (False, True):
            ops.FUSE_LN_BWD = fuse
            ops._CrossAttnBlock.backward = staticmethod(recording) if not fuse else orig
            mem = mem0.clone().requires_grad_(True)
            memp = memp0.clone().requires_grad_(True)
            ops.begin_pass()
            hs, _, _ = tr.decode(mem, memp, B, S, kpm, tgt, tm, torch.bfloat16)
            loss = (hs.float() * w_hs).sum()
            if extra_use:
                loss = loss + (mem.float() * w_x).sum()
            loss.backward()
            torch.cuda.synchronize()
            res[fuse] = (memp.grad.float().clone(), mem.grad.float().clone())
    finally:
        ops.FUSE_LN_BWD = True
        ops._CrossAttnBlock.backward = orig
    assert len(contrib) == 6
    extra = w_x.to(torch.bfloat16).float() if extra_use else torch.zeros_like(w_x)
    for i, what in enumerate(("dmem_pos", "dmem")):
        parts = [c[i] for c in contrib]
        s = torch.stack(parts).sum(0) + (extra if i == 1 else 0)
        mag = torch.stack([p.abs() for p in parts]).sum(0) + (extra.abs() if i == 1 else 0)
        for fuse in (True, False):
            got = res[fuse][i]
            assert torch.isfinite(got).all()
            # <= 7 adds, each rounding the running sum to bf16 (2^-9 relative): 2^-6 of the
            # element's absolute-sum is a 2x margin
            bad = ((got - s).abs() > 2.0 ** -6 * mag + 1e-6).sum().item()
            assert bad == 0, (what, fuse, bad, (got - s).abs().max().item())
            e = ((got - s).norm() / s.norm()).item()
            assert e < 1e-2, (what, fuse, e)


def test_deferred_weight_gradients_match_per_block_launches():
    """bf16 training with FusedAdamW's gradient arena: the transformer blocks' weight / bias /
    LayerNorm-parameter gradients are queued and run as ONE retr_linear_wgrad_batch launch at
    the end of backward (ops.WGRAD_DEFER, flushed by autograd's final callback -- no explicit
    flush here) instead of one grouped split-K launch + slab sum per block.  Against the
    per-block path (which at these token counts does not split the reduction either): every
    gradient bitwise equal, one flush per backward and nothing left queued.  (Split-K vs the
    unsplit batch at the full token counts: tests/test_gpu_kernels.py::test_wgrad_batch_*.)"""
    from retr_amd import ops
    from retr_amd.optim import FusedAdamW
    cfg = make_config(backbone="ResNet18", hidden=256, layers=(2, 2), vocab=1000, max_pos=16,
                      ffn=512, dtype="bf16", dropout=0.1)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=4))
    model.to(DEV).train()
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    images, mask = synthetic_images(2, 64, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(2, 16, 1000, seed=2)
    s = NestedTensor(images.to(DEV), mask.to(DEV))
    ctr = ops._seed_state["ctr"]
    res = []
    try:
        for defer in (True, False):
            ops.WGRAD_DEFER = defer
            ops._seed_state["ctr"] = ctr
            f0 = ops.WGRAD_STATS["flushes"]
            opt.zero_grad(set_to_none=True)
            out = model(s, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
            loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
            loss.backward()
            assert ops.wgrad_pending() == 0
            torch.cuda.synchronize()
            res.append(({n: p.grad.detach().clone() for n, p in model.named_parameters()
                         if p.grad is not None}, ops.WGRAD_STATS["flushes"] - f0, loss.item()))
    finally:
        ops.WGRAD_DEFER = True
    (g1, nf1, l1), (g0, nf0, l0) = res
    assert l1 == l0
    assert nf1 == 1 and nf0 == 0, (nf1, nf0)
    assert g1.keys() == g0.keys() and len(g1) > 0
    # at these token counts (< 512 per block) the per-block path does not split the reduction
    # either, so both are the same single fp32 chain per element: bitwise equal everywhere but
    # in the MLP head (deferred: the batch kernel, biases as its all-ones MFMA; per-launch: the
    # single-problem wgrad kernel and a fixed-order column sum -- the same sums in another order)
    for n in g1:
        if n.startswith("mlp."):
            e = ((g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-30)).item()
            assert e < 1e-5, (n, e)
        else:
            assert torch.equal(g1[n], g0[n]), n


def test_grouped_conv_weight_gradients_match_per_conv_launches():
    """bf16 ResNet-50 backbone backward: the queued conv weight gradients run as grouped
    launches (resnet.CONV_WGRAD_GROUP) against one split-K launch + unpack per conv: every
    trainable backbone weight gradient within fp32 reassociation of the slice sums (rel 1e-5),
    nothing else changed (the data-gradient chain is the same kernels: input_proj and the
    transformer bitwise equal)."""
    from retr_amd import resnet
    cfg = make_config(backbone="ResNet50", hidden=64, layers=(1, 1), vocab=1000, max_pos=16,
                      ffn=128, dtype="bf16", dropout=0.0)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=6))
    model.to(DEV).train()
    images, mask = synthetic_images(2, 256, seed=3, pad_band=True)
    caps, cap_mask = synthetic_captions(2, 16, 1000, seed=4)
    s = NestedTensor(images.to(DEV), mask.to(DEV))
    res = []
    try:
        for grp in (True, False):
            resnet.CONV_WGRAD_GROUP = grp
            st0 = dict(resnet.CONV_WGRAD_STATS)
            model.zero_grad(set_to_none=True)
            out = model(s, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
            loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
            loss.backward()
            torch.cuda.synchronize()
            res.append(({n: p.grad.detach().clone() for n, p in model.named_parameters()
                         if p.grad is not None},
                        resnet.CONV_WGRAD_STATS["grouped"] - st0["grouped"]))
    finally:
        resnet.CONV_WGRAD_GROUP = True
    (g1, n1), (g0, n0) = res
    assert n1 > 20 and n0 == 0, (n1, n0)
    assert g1.keys() == g0.keys()
    nb = 0
    for n in g1:
        if n.startswith("backbone"):
            r = ((g1[n] - g0[n]).double().norm() / (g0[n].double().norm() + 1e-30)).item()
            assert r < 1e-5, (n, r)
            nb += 1
        else:
            assert torch.equal(g1[n], g0[n]), n
    assert nb > 20


def test_next_layernorm_in_ffn_epilogue_matches_separate_launch():
    """The FFN down-projection's epilogue also produces the LayerNorm that reads its output
    next (ops.FUSE_LN_NEXT: the following block's pre-norm, the encoder's final LN(x) / LN(x) +
    pos, the decoder's final norm) -- the consumer takes the tagged result instead of launching
    its own LayerNorm.  Loss and every gradient bitwise equal to the separate-launch path, and
    every FFN output was consumed that way (2 + 2 layers: 4 hits per forward)."""
    from retr_amd import ops
    cfg = make_config(backbone="ResNet18", hidden=256, layers=(2, 2), vocab=1000, max_pos=16,
                      ffn=512, dtype="bf16", dropout=0.1)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=6))
    model.to(DEV).train()
    images, mask = synthetic_images(2, 64, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(2, 16, 1000, seed=2)
    s = NestedTensor(images.to(DEV), mask.to(DEV))
    ctr = ops._seed_state["ctr"]
    res = []
    try:
        for fuse in (True, False):
            ops.FUSE_LN_NEXT = fuse
            ops._seed_state["ctr"] = ctr
            h0 = ops.LN_NEXT_STATS["hit"]
            model.zero_grad(set_to_none=True)
            out = model(s, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
            loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
            loss.backward()
            torch.cuda.synchronize()
            res.append(({n: p.grad.detach().clone() for n, p in model.named_parameters()
                         if p.grad is not None}, ops.LN_NEXT_STATS["hit"] - h0, loss.item(),
                        out.detach().clone()))
    finally:
        ops.FUSE_LN_NEXT = True
    (g1, h1, l1, o1), (g0, h0, l0, o0) = res
    assert h1 == 4 and h0 == 0, (h1, h0)
    assert l1 == l0 and torch.equal(o1, o0)
    assert g1.keys() == g0.keys() and len(g1) > 0
    for n in g1:
        assert torch.equal(g1[n], g0[n]), n


def test_deferred_position_gradients_match_per_block_launches():
    """The decoder blocks' query-position gradient contributions queued and summed by one
    retr_pos_grad_multi launch at the weight-gradient flush (ops.POS_DEFER, FusedAdamW arena)
    against one retr_pos_grad launch per block: every gradient bitwise equal."""
    from retr_amd import ops
    from retr_amd.optim import FusedAdamW
    cfg = make_config(backbone="ResNet18", hidden=256, layers=(2, 2), vocab=1000, max_pos=16,
                      ffn=512, dtype="bf16", dropout=0.1)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=8))
    model.to(DEV).train()
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    images, mask = synthetic_images(2, 64, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(2, 16, 1000, seed=2)
    s = NestedTensor(images.to(DEV), mask.to(DEV))
    ctr = ops._seed_state["ctr"]
    res = []
    try:
        for defer in (True, False):
            ops.POS_DEFER = defer
            ops._seed_state["ctr"] = ctr
            opt.zero_grad(set_to_none=True)
            out = model(s, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
            loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
            loss.backward()
            assert not ops._POSQ
            torch.cuda.synchronize()
            # the table's 12 query-position contributions and the embedding's own sum meet in
            # ONE arena buffer that autograd adopts (round 4 lost the queued part: autograd
            # cloned the buffer before the queued sums were written)
            foreign = [n for n, p in model.named_parameters() if p.grad is not None
                       and p.grad.data_ptr() != p._retr_grad_view.data_ptr()]
            assert not foreign, foreign
            res.append({n: p.grad.detach().clone() for n, p in model.named_parameters()
                        if p.grad is not None})
    finally:
        ops.POS_DEFER = True
    g1, g0 = res
    assert g1.keys() == g0.keys()
    assert any("position_embeddings" in n for n in g1)
    for n in g1:
        assert torch.equal(g1[n], g0[n]), n


def test_position_table_gradient_has_every_contribution():
    """position_embeddings.weight is read twice by the reference (DecoderEmbeddings,
    transformer_modules.py:118-127, and as the decoder's query_pos, ConcatTransformer.py:64-65):
    its gradient through the default bf16 FusedAdamW path (deferred query-position sums) equals
    the sum of both uses, computed here by differentiating the two uses separately -- a
    missing contribution (round 4's bug) is an O(1) relative error, far above bf16 noise."""
    from retr_amd import ops
    from retr_amd.optim import FusedAdamW
    cfg = make_config(backbone="ResNet18", hidden=256, layers=(2, 2), vocab=1000, max_pos=16,
                      ffn=512, dtype="bf16", dropout=0.0)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=9))
    model.to(DEV).train()
    opt = FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)
    images, mask = synthetic_images(2, 64, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(2, 16, 1000, seed=2)
    s = NestedTensor(images.to(DEV), mask.to(DEV))
    pw = model.transformer.embeddings.position_embeddings.weight

    def run():
        opt.zero_grad(set_to_none=True)
        out = model(s, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
        loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        return pw.grad.detach().clone()

    full = run()
    # the per-block launches (POS_DEFER off) give the same bits
    ops.POS_DEFER = False
    try:
        ref = run()
    finally:
        ops.POS_DEFER = True
    assert torch.equal(full, ref)
    # embedding-only gradient: the same forward with the decoder blocks' query positions
    # detached (decode() calls ops.self_attn_block / ops.cross_attn_block at run time)
    saved = ops.self_attn_block, ops.cross_attn_block

    def sab(sa, y, qpos, *a, **k):
        return saved[0](sa, y, qpos.detach() if qpos is pw else qpos, *a, **k)

    def cab(ca, y, qpos, *a, **k):
        return saved[1](ca, y, qpos.detach() if qpos is pw else qpos, *a, **k)
    ops.self_attn_block, ops.cross_attn_block = sab, cab
    try:
        emb_only = run()
    finally:
        ops.self_attn_block, ops.cross_attn_block = saved
    # query-position-only gradient: the embedding reads a detached table
    saved_e = ops.embed_ln

    def el(emb, caps_, training, shared=False):
        w = emb.position_embeddings.weight
        emb.position_embeddings.weight = torch.nn.Parameter(w.detach(), requires_grad=False)
        try:
            return saved_e(emb, caps_, training, shared=False)
        finally:
            emb.position_embeddings.weight = w
    ops.embed_ln = el
    try:
        q_only_g = run()
    finally:
        ops.embed_ln = saved_e
    both = emb_only.double() + q_only_g.double()
    e = ((full.double() - both).norm() / both.norm()).item()
    assert e < 1e-5, e
    # each use really contributes, far above the 1e-5 bound (else the test would be vacuous):
    # at this size the 4 query-position uses are ~2% of the table's gradient norm
    assert q_only_g.norm() > 1e-3 * both.norm() and emb_only.norm() > 1e-3 * both.norm()


def test_deferred_weight_used_twice_flushes_before_second_contribution():
    """A parameter with a deferred (queued) weight gradient that gets a second contributor in
    the same backward: autograd adds the two, reading the first (arena) buffer, so the queue
    must have run first (optim.REUSE_HOOK -> ops._on_grad_reuse).  The MLP head applied twice
    in one graph, FusedAdamW arena, bf16: every gradient equals the immediate-launch path
    (rel 1e-5: batch vs single-problem kernels) and the sum of the two uses' gradients taken one
    use per backward, and the hook fired."""
    from retr_amd import ops
    from retr_amd.models.caption import MLP
    from retr_amd.optim import FusedAdamW
    torch.manual_seed(0)
    B, T, C, V = 2, 16, 64, 1000
    mlp = MLP(C, 128, V, 3).to(DEV)
    opt = FusedAdamW(list(mlp.parameters()), lr=1e-4)
    hs = [torch.randn(B * T, C, device=DEV).to(torch.bfloat16) for _ in range(2)]
    wts = [torch.randn(B, T, V, device=DEV) for _ in range(2)]
    res = []
    try:
        for defer in (True, False):
            ops.HEAD_WGRAD_DEFER = defer
            opt.zero_grad(set_to_none=True)
            ops.begin_pass()
            r0 = ops.GRAD_REUSE_STATS["flushes"]
            loss = sum((ops.mlp_head(mlp, h, B, T, torch.bfloat16).float() * w).sum()
                       for h, w in zip(hs, wts))
            loss.backward()
            torch.cuda.synchronize()
            res.append(({n: p.grad.detach().clone() for n, p in mlp.named_parameters()},
                        ops.GRAD_REUSE_STATS["flushes"] - r0))
    finally:
        ops.HEAD_WGRAD_DEFER = True
    (g1, f1), (g0, f0) = res
    assert f1 >= 1 and f0 == 0, (f1, f0)
    # every contribution: the sum of the two uses' gradients, each from its own backward (one
    # use per pass, so nothing is reused or queued twice) -- equal up to the order of the final
    # fp32 add; a lost use would be an O(1) relative error
    single = []
    for h, w in zip(hs, wts):
        opt.zero_grad(set_to_none=True)
        ops.begin_pass()
        (ops.mlp_head(mlp, h, B, T, torch.bfloat16).float() * w).sum().backward()
        torch.cuda.synchronize()
        single.append({n: p.grad.detach().clone() for n, p in mlp.named_parameters()})
    for n in g1:
        e = ((g1[n] - g0[n]).double().norm() / g0[n].double().norm()).item()
        assert e < 1e-5, (n, e)
        r = single[0][n].double() + single[1][n].double()
        e = ((g1[n].double() - r).norm() / r.norm()).item()
        assert e < 1e-5, (n, e)


def test_grouped_conv_wgrad_tile_layouts_bitwise():
    """The grouped conv weight-gradient launches under every tile layout (RETR_TUNE_CW_WAVES:
    128 x 128 on 4 or 8 waves, 128 x 256 on 8 waves) give bitwise-equal gradients: the same
    K-slices, each output element's MFMA chain over the slice in the same order."""
    from retr_amd import _lib, resnet
    cfg = make_config(backbone="ResNet50", hidden=64, layers=(1, 1), vocab=1000, max_pos=16,
                      ffn=128, dtype="bf16", dropout=0.0)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=6))
    model.to(DEV).train()
    images, mask = synthetic_images(2, 256, seed=3, pad_band=True)
    caps, cap_mask = synthetic_captions(2, 16, 1000, seed=4)
    s = NestedTensor(images.to(DEV), mask.to(DEV))
    res = []
    try:
        resnet.CONV_WGRAD_GROUP = True
        for layout in (0, 1, 2, 3):
            _lib.load().retr_tune(29, layout)
            model.zero_grad(set_to_none=True)
            out = model(s, caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))
            crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV)).backward()
            torch.cuda.synchronize()
            res.append({n: p.grad.detach().clone() for n, p in model.named_parameters()
                        if p.grad is not None and n.startswith("backbone")})
    finally:
        _lib.load().retr_tune(29, 0)
    assert len(res[0]) > 20
    for r in res[1:]:
        for n in res[0]:
            assert torch.equal(r[n], res[0][n]), n
