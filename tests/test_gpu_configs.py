"""BASELINE.json configurations exercised on the GPU.

* cfg2 (R50 6/6 d256, 640x640): fp32 parity mode at batch 1 against the CPU oracle (logits /
  loss within 1e-3, gradient norms within 2e-3); the benchmarked bf16 path at batch 2 against
  the CPU oracle and at the benchmarked batch 16 (dropout 0.1 and 0) against the fp32 HIP
  model: every trainable gradient within BF16_GRAD_REL (relative L2).
* cfg4 (R101 6/6 d512 nhead 8, 800x800): fp32 at batch 1 against the oracle.
* cfg5 (R50 dilation=True 224x224, 6/6 d256, V 30522, T 128): greedy ids at batch 64 in bf16
  (hipGraph replay == eager launches, == the full-recompute reference algorithm on the GPU
  wherever the recompute's top-2 logit margin is above bf16 rounding), and fp32 at batch 2
  bit-exact against the oracle's reference algorithm.
* cfg4 per-GPU slice at full size (batch 8, 800x800, bf16): fwd + bwd, every trainable
  gradient vs the fp32 HIP model.
* cfg5 fp32 at batch 64: 4 rows' ids vs the CPU oracle's reference algorithm.
cfg3 is cfg2 under data parallelism (tests/test_ddp_*.py, tests/test_gpu_ddp.py); cfg1 is in
test_gpu_model.py.
"""
import pytest
import torch

from oracle import model as orc
from retr_amd.eval_utils.decode import IncrementalGreedy, greedy, greedy_reference_algorithm
from retr_amd.models.caption import build_model
from retr_amd.models.utils import NestedTensor
from retr_amd.synthetic import synthetic_captions, synthetic_images, synthetic_state_dict
from tests.helpers import make_config

pytestmark = pytest.mark.gpu
DEV = "cuda"

CFG2 = dict(backbone="ResNet50", dilation=False, hidden=256, layers=(6, 6), vocab=30522,
            max_pos=128, ffn=2048)
CFG4 = dict(backbone="ResNet101", dilation=False, hidden=512, layers=(6, 6), vocab=30522,
            max_pos=128, ffn=2048)
CFG5 = dict(backbone="ResNet50", dilation=True, hidden=256, layers=(6, 6), vocab=30522,
            max_pos=128, ffn=2048)


def _model(kw, dtype, dropout=0.0):
    cfg = make_config(dtype=dtype, dropout=dropout, **kw)
    model, crit = build_model(cfg)
    sd = synthetic_state_dict(model, seed=42)
    model.load_state_dict(sd)
    return cfg, model.to(DEV), crit, sd


def _max_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _parity_vs_oracle(kw, size, B):
    cfg, model, crit, sd = _model(kw, "fp32")
    images, mask = synthetic_images(B, size, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=2)
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
    assert _max_rel(out, lo) < 1e-3
    assert abs(loss.item() - loss_o.item()) <= 1e-3 * abs(loss_o.item())
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        go = sdo[n].grad
        denom = go.norm().item()
        if denom == 0:
            continue
        e = ((p.grad.double().cpu() - go.double()).norm() / denom).item()
        assert e < 2e-3, (n, e)
    return loss.item()


def test_cfg2_fp32_batch1_matches_oracle():
    _parity_vs_oracle(CFG2, 640, 1)


def test_cfg4_fp32_batch1_matches_oracle():
    _parity_vs_oracle(CFG4, 800, 1)


# Per-tensor bound of the bf16 path against fp32 (oracle or the fp32 HIP model): relative L2
# error of EVERY trainable gradient.  bf16 operands carry 8 significant bits (2^-9 = 2e-3
# relative per rounding); errors compound through ~100 layers of backward, so the bound is an
# order of magnitude above one rounding -- and an order below what one wrong weight-gradient
# kernel (a dropped split, a wrong tap, a transposed tile) produces (>= 0.3).
BF16_GRAD_REL = 3e-2


def _grad_errors(model, ref):
    """{name: relative L2 error of p.grad vs ref[name]} over every trainable parameter with a
    nonzero reference gradient (ref: fp32 tensors on any device)."""
    errs = {}
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        assert p.grad is not None and torch.isfinite(p.grad).all(), n
        r = ref[n].to(p.grad.device, torch.float64)
        d = r.norm().item()
        if d == 0:
            assert p.grad.abs().max().item() == 0, n
            continue
        errs[n] = ((p.grad.double() - r).norm() / d).item()
    return errs


# LayerNorm gamma / beta gradients are column sums over every token row (2048-6400 rows) of
# terms that largely cancel (sum_r dy_r * xhat_r): the sum's relative error exceeds the
# per-element bf16 error by the cancellation ratio, so they get their own, looser bound.
BF16_LN_GRAD_REL = 1e-1


def _is_norm(name):
    return ".norm." in name or "LayerNorm" in name or name.startswith("transformer.decoder.norm")


def _assert_grads(errs, bound, what, ln_bound=BF16_LN_GRAD_REL):
    worst = sorted(((n, e) for n, e in errs.items() if not _is_norm(n)), key=lambda kv: -kv[1])
    worst_ln = sorted(((n, e) for n, e in errs.items() if _is_norm(n)), key=lambda kv: -kv[1])
    msg = f"{what}: worst per-tensor gradient errors {worst[:6]}; LayerNorm {worst_ln[:4]}"
    print(msg)
    assert worst and worst[0][1] < bound, msg
    assert not worst_ln or worst_ln[0][1] < ln_bound, msg


def _seeded_step(model, crit, images, mask, caps, cap_mask, seed_ctr=0, seed_base=None):
    """forward + CE + backward with the dropout seed stream reset: every op draws the same
    per-op seed and the same device step seed, so the fp32 and bf16 models drop the same
    units (one keep(seed, index) hash on both paths)."""
    from retr_amd import ops
    ops._seed_state["ctr"] = seed_ctr
    if seed_base is not None:
        ops.seed_base().fill_(seed_base)
    model.train()
    out = model(NestedTensor(images.to(DEV), mask.to(DEV)), caps[:, :-1].to(DEV),
                cap_mask[:, :-1].to(DEV))
    loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
    loss.backward()
    return out, loss


def _attach_arena(model):
    """The benchmarked optimizer (FusedAdamW): every trainable parameter moves into its arena,
    so the backward writes weight gradients into arena slots and the deferred paths run
    (ops.WGRAD_DEFER: the transformer + head weight gradients as one batched launch,
    ops.POS_DEFER: the query-position sums, resnet.CONV_WGRAD_GROUP)."""
    from retr_amd.optim import FusedAdamW
    return FusedAdamW([p for p in model.parameters() if p.requires_grad], lr=1e-4)


def _assert_adopted(model):
    """Every trainable gradient IS its arena slot: autograd adopted the buffer the kernels wrote
    (no second contribution added outside it, no clone taken before a deferred sum landed)."""
    foreign = [n for n, p in model.named_parameters() if p.requires_grad
               and (p.grad is None or p.grad.data_ptr() != p._retr_grad_view.data_ptr())]
    assert not foreign, foreign


def _defer_counters():
    from retr_amd import ops, resnet
    return (ops.WGRAD_STATS["flushes"], ops.WGRAD_STATS["problems"],
            resnet.CONV_WGRAD_STATS["grouped"])


@pytest.mark.parametrize("dropout,arena", [(0.0, False), (0.1, False), (0.1, True)])
def test_cfg2_bf16_full_batch_step(dropout, arena):
    """The benchmarked shape (batch 16, 640x640, bf16 operands, dropout 0.1 as timed and 0.0)
    forward + backward against the fp32 HIP model (exact-f32 MFMA; the fp32 path is pinned to
    the CPU oracle at cfg2 / cfg4 batch 1 above) on the same weights, inputs and dropout
    masks: loss within 1e-2 and EVERY trainable gradient within BF16_GRAD_REL (relative L2).
    ``arena``: with the benchmarked FusedAdamW attached, so the gradients come through the
    deferred weight-gradient batch, the queued position sums and the grouped conv weight
    gradients, read from the arena before any step().  Reference step: engine.py:70-80."""
    B = 16
    images, mask = synthetic_images(B, 640, seed=3)
    _, m32, crit, _ = _model(CFG2, "fp32", dropout=dropout)
    cfg, m16, _, _ = _model(CFG2, "bf16", dropout=dropout)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=4)
    _, l32 = _seeded_step(m32, crit, images, mask, caps, cap_mask, 1000, 12345)
    ref = {n: p.grad.detach().clone() for n, p in m32.named_parameters() if p.requires_grad}
    l32 = l32.item()
    del m32
    torch.cuda.empty_cache()
    opt = _attach_arena(m16) if arena else None
    c0 = _defer_counters()
    _, l16 = _seeded_step(m16, crit, images, mask, caps, cap_mask, 1000, 12345)
    c1 = _defer_counters()
    l16 = l16.item()
    assert torch.isfinite(torch.tensor([l16, l32])).all()
    assert abs(l16 - l32) <= 1e-2 * abs(l32), (l16, l32)
    if arena:
        _assert_adopted(m16)
        # one batched transformer + head launch (~90 problems at 6/6), grouped conv wgrads
        assert c1[0] - c0[0] >= 1 and c1[1] - c0[1] >= 80 and c1[2] - c0[2] > 40, (c0, c1)
    errs = _grad_errors(m16, ref)
    assert len(errs) >= 230, len(errs)
    _assert_grads(errs, BF16_GRAD_REL, f"cfg2 bf16 B=16 dropout {dropout} arena {arena}")
    del opt


@pytest.mark.parametrize("arena", [False, True])
def test_cfg2_bf16_batch2_vs_oracle(arena):
    """The bf16 training path at cfg2's image size (640x640, R50 6/6 d256; batch 2) against the
    CPU oracle directly: logits within 2e-2 of the oracle's scale, loss within 1e-2, every
    trainable gradient within BF16_GRAD_REL.  ``arena``: through the benchmarked FusedAdamW
    arena (deferred / batched weight and position gradients), gradients read before step().
    Reference: engine.py:70-80 on models/caption.py:23-47."""
    B = 2
    cfg, model, crit, sd = _model(CFG2, "bf16")
    images, mask = synthetic_images(B, 640, seed=21, pad_band=True)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=22)
    opt = _attach_arena(model) if arena else None
    out, loss = _seeded_step(model, crit, images, mask, caps, cap_mask)
    if arena:
        _assert_adopted(model)
        del opt
    trainable = {n for n, p in model.named_parameters() if p.requires_grad}
    sdo = {k: (v.clone().requires_grad_(True) if k in trainable else v) for k, v in sd.items()}
    lo = orc.caption_forward(sdo, cfg, images, mask, caps[:, :-1], cap_mask[:, :-1])
    loss_o = orc.caption_loss(lo, caps[:, 1:])
    loss_o.backward()
    assert out.shape == lo.shape
    assert _max_rel(out.float(), lo) < 2e-2
    assert abs(loss.item() - loss_o.item()) <= 1e-2 * abs(loss_o.item())
    errs = _grad_errors(model, {n: sdo[n].grad for n in trainable})
    _assert_grads(errs, BF16_GRAD_REL, "cfg2 bf16 B=2 vs oracle")


def test_cfg2_graphed_step_gradients_vs_fp32():
    """The timed step itself: bench.py's GraphedTrainStep (cfg2, batch 16, bf16, dropout 0.1,
    FusedAdamW arena, every deferral on) captured and replayed once with consume mode off and
    no clipping, so the replay's gradients stay in the arena -- against the fp32 HIP model's
    eager backward on the same weights (the replay runs at the restored pre-warm-up weights),
    inputs and dropout masks (the capture's per-op seeds and the device step seed bumped
    once): loss within 1e-2, EVERY trainable gradient within BF16_GRAD_REL.
    Reference: engine.py:70-83."""
    from retr_amd import ops
    from retr_amd.engine import GraphedTrainStep
    B = 16
    images, mask = synthetic_images(B, 640, seed=5)
    cfg, m16, crit, _ = _model(CFG2, "bf16", dropout=0.1)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=6)
    opt = _attach_arena(m16)
    step = GraphedTrainStep(m16, crit, opt, max_norm=0.0, consume=False)
    box = {}
    cap = step._capture

    def rec():
        box["ctr"] = ops._seed_state["ctr"]
        cap()
    step._capture = rec
    base = int(ops.seed_base().item())
    loss16 = float(step((NestedTensor(images.to(DEV), mask.to(DEV)),), caps.to(DEV),
                        cap_mask.to(DEV)))
    torch.cuda.synchronize()
    names = [n for n, p in m16.named_parameters() if p.requires_grad]
    g16 = {n: p._retr_grad_view.detach().clone() for n, p in m16.named_parameters()
           if p.requires_grad}
    del step, opt, m16
    torch.cuda.empty_cache()
    _, m32, _, _ = _model(CFG2, "fp32", dropout=0.1)
    ops.seed_base().fill_(base)
    ops.bump_seed()                      # forward_backward's bump, replayed inside the graph
    _, l32 = _seeded_step(m32, crit, images, mask, caps, cap_mask, box["ctr"], None)
    l32 = l32.item()
    assert abs(loss16 - l32) <= 1e-2 * abs(l32), (loss16, l32)

    class _G:                            # _grad_errors reads p.grad / named_parameters
        def __init__(self, g):
            self.g = g

        def named_parameters(self):
            for n in names:
                yield n, type("P", (), {"requires_grad": True, "grad": self.g[n]})()
    ref = {n: p.grad.detach() for n, p in m32.named_parameters() if p.requires_grad}
    errs = _grad_errors(_G(g16), ref)
    assert len(errs) >= 230, len(errs)
    _assert_grads(errs, BF16_GRAD_REL, "cfg2 graphed step (one replay) vs fp32")


def _recompute_margins(model, samples, ids):
    """Top-2 margin of the full-recompute logits at every decoded position."""
    with torch.no_grad():
        cm = ids == 0
        cm[:, 0] = False
        out = model(samples[0], ids, cm)
        top2 = out.float().topk(2, dim=-1).values
        return (top2[..., 0] - top2[..., 1])


def test_cfg5_greedy_bf16_batch64():
    cfg, model, _, _ = _model(CFG5, "bf16")
    model.eval()
    B, T = 64, cfg.max_position_embeddings
    images, mask = synthetic_images(B, 224, seed=7)
    samples = [NestedTensor(images.to(DEV), mask.to(DEV))]
    ids = greedy(samples, model, max_len=T, bos_token=101, eos_token=102)        # hipGraphs
    ids_eager = IncrementalGreedy(model, use_graphs=False)(samples[0], T, 101, 102)
    assert torch.equal(ids, ids_eager)            # graph replay == eager launches, bitwise
    ids2 = greedy(samples, model, max_len=T, bos_token=101, eos_token=102)       # replayed
    assert torch.equal(ids, ids2)
    ids_full = greedy_reference_algorithm(samples, model, T, 101, 102)
    # the recompute runs the tiled training attention (different reduction order than the
    # single-query decode kernel), so ids may only differ after a position whose top-2 logit
    # margin is within bf16 rounding; everything before the first such tie must agree
    margins = _recompute_margins(model, samples, ids_full)
    for b in range(B):
        diff = (ids[b] != ids_full[b]).nonzero()
        if diff.numel() == 0:
            continue
        j = int(diff[0])               # first differing column: decided at step j-1
        assert float(margins[b, j - 1]) < 0.05, (b, j, float(margins[b, j - 1]))
    # (random weights give near-uniform next-token distributions, so near-ties are common and
    # most rows eventually diverge in bf16; the fp32 test below is the bit-exact one)


def test_cfg5_greedy_fp32_batch2_bit_exact_vs_oracle():
    cfg, model, _, sd = _model(CFG5, "fp32")
    model.eval()
    B, T = 2, cfg.max_position_embeddings
    images, mask = synthetic_images(B, 224, seed=8, pad_band=True)
    ids = greedy([NestedTensor(images.to(DEV), mask.to(DEV))], model, max_len=T,
                 bos_token=101, eos_token=102)
    with torch.no_grad():
        ids_o = orc.greedy(lambda c, m: orc.caption_forward(sd, cfg, images, mask, c, m), B, T,
                           101, 102)
    assert torch.equal(ids.cpu(), ids_o)


def test_cfg4_bf16_full_slice_step():
    """cfg4's per-GPU slice at full size (R101 6/6 d512 nhead 8, 800x800, batch 8, bf16):
    forward + backward through the hd = 64 attention path at S = 625 against the fp32 HIP
    model on the same weights and inputs: loss within 1e-2, EVERY trainable gradient within
    BF16_GRAD_REL.  Reference shapes: models/backbone.py:86-91,
    models/ConcatTransformer.py:259-269."""
    B = 8
    images, mask = synthetic_images(B, 800, seed=11)
    _, m32, crit, _ = _model(CFG4, "fp32")
    caps, cap_mask = synthetic_captions(B, 128, 30522, seed=12)
    _, l32 = _seeded_step(m32, crit, images, mask, caps, cap_mask)
    ref = {n: p.grad.detach().clone() for n, p in m32.named_parameters() if p.requires_grad}
    l32 = l32.item()
    del m32
    torch.cuda.empty_cache()
    cfg, m16, _, _ = _model(CFG4, "bf16")
    out, l16 = _seeded_step(m16, crit, images, mask, caps, cap_mask)
    assert out.shape == (B, 128, 30522)
    l16 = l16.item()
    assert torch.isfinite(torch.tensor([l16, l32])).all()
    assert abs(l16 - l32) <= 1e-2 * abs(l32), (l16, l32)
    errs = _grad_errors(m16, ref)
    _assert_grads(errs, BF16_GRAD_REL, "cfg4 bf16 B=8")


def test_cfg5_greedy_fp32_batch64_graphs_eager_recompute_bitwise():
    """Parity mode (fp32, exact-f32 MFMA) at the decode config's batch: hipGraph replay ==
    eager launches == the reference's full-recompute algorithm (decode.py:53-81, 127 full
    forwards) on the GPU, token for token.  (The B=2 test above pins the same ids to the CPU
    oracle.)"""
    cfg, model, _, _ = _model(CFG5, "fp32")
    model.eval()
    B, T = 64, cfg.max_position_embeddings
    images, mask = synthetic_images(B, 224, seed=9, pad_band=True)
    samples = [NestedTensor(images.to(DEV), mask.to(DEV))]
    ids = greedy(samples, model, max_len=T, bos_token=101, eos_token=102)        # hipGraphs
    ids_eager = IncrementalGreedy(model, use_graphs=False)(samples[0], T, 101, 102)
    assert torch.equal(ids, ids_eager)
    ids_full = greedy_reference_algorithm(samples, model, T, 101, 102)
    diff = (ids != ids_full).any(1).nonzero().flatten().tolist()
    if diff:
        margins = _recompute_margins(model, samples, ids_full)
        info = []
        for b in diff:
            j = int((ids[b] != ids_full[b]).nonzero()[0])
            info.append((b, j, float(margins[b, j - 1])))
        raise AssertionError(f"rows differing from the reference algorithm (row, first "
                             f"column, top-2 margin there): {info}")


def test_cfg5_greedy_fp32_batch64_rows_vs_oracle():
    """The decode config's real batch (cfg5, fp32 parity mode, B = 64): the ids of 4 of its
    rows (first, last and two inside) equal the CPU oracle's reference algorithm
    (decode.py:53-81: a full forward per token) run on those rows alone -- rows of a batch are
    independent bit-for-bit, so this pins the full-batch ids without 64
    oracle decodes."""
    cfg, model, _, sd = _model(CFG5, "fp32")
    model.eval()
    B, T = 64, cfg.max_position_embeddings
    images, mask = synthetic_images(B, 224, seed=9, pad_band=True)
    ids = greedy([NestedTensor(images.to(DEV), mask.to(DEV))], model, max_len=T,
                 bos_token=101, eos_token=102).cpu()
    rows = [0, 17, 42, 63]
    with torch.no_grad():
        ids_o = orc.greedy(lambda c, m: orc.caption_forward(sd, cfg, images[rows], mask[rows],
                                                            c, m), len(rows), T, 101, 102)
    assert torch.equal(ids[rows], ids_o), [(r, int((ids[r] != ids_o[i]).nonzero()[0]))
                                           for i, r in enumerate(rows)
                                           if not torch.equal(ids[r], ids_o[i])]
