"""FusedAdamW (retr_amd/optim.py + csrc/optim.hip) against torch.optim.AdamW + clip_grad_norm_
(the reference's optimizer step, main.py:39-41 / engine.py:80-83), and the gradient arena that
the backward Functions write into."""
import copy

import pytest
import torch

from retr_amd.models.utils import NestedTensor
from retr_amd.optim import FusedAdamW
from tests.helpers import make_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(7, 13), (256,), (3, 5, 2), (1,), (1000,), (64, 33)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in shapes]


@pytest.mark.parametrize("max_norm", [0.0, 0.5, 1e6])
def test_fused_adamw_matches_torch(max_norm):
    ref = _params(0)
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]

    def groups(ps):
        return [{"params": ps[:3]}, {"params": ps[3:], "lr": 3e-3, "weight_decay": 0.0}]
    opt_r = torch.optim.AdamW(groups(ref), lr=1e-2, weight_decay=1e-2, foreach=False)
    opt_m = FusedAdamW(groups(mine), lr=1e-2, weight_decay=1e-2)
    g = torch.Generator().manual_seed(1)
    for it in range(4):
        grads = [torch.randn(p.shape, generator=g).to(DEV) * (it + 1) for p in ref]
        for k, (pr, pm, gr) in enumerate(zip(ref, mine, grads)):
            skip = it == 2 and k in (1, 4)          # parameters without a gradient this step
            pr.grad = None if skip else gr.clone()
            pm.grad = None if skip else gr.clone()  # foreign gradients: copied into the arena
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_([p for p in ref if p.grad is not None], max_norm,
                                           foreach=False)
        opt_r.step()
        opt_m.step(max_norm=max_norm)
        if it == 1:                                  # lr schedule change between steps
            for o in (opt_r, opt_m):
                o.param_groups[0]["lr"] *= 0.5
        for pr, pm in zip(ref, mine):
            assert _rel(pm.detach(), pr.detach()) < 2e-6
            if pr.grad is not None:
                assert _rel(pm.grad, pr.grad) < 2e-6     # clipped gradients written back
            sr, sm = opt_r.state[pr], opt_m.state[pm]
            if sr:
                assert _rel(sm["exp_avg"], sr["exp_avg"]) < 2e-6
                assert _rel(sm["exp_avg_sq"], sr["exp_avg_sq"]) < 2e-6


def test_fused_adamw_state_dict_roundtrip():
    ps = _params(2)
    opt = FusedAdamW([{"params": ps}], lr=1e-3)
    for p in ps:
        p.grad = torch.ones_like(p)
    opt.step()
    sd = copy.deepcopy(opt.state_dict())
    ps2 = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt2 = FusedAdamW([{"params": ps2}], lr=1e-3)
    opt2.load_state_dict(sd)
    for p, q in ((p, q) for p, q in zip(ps, ps2)):
        assert torch.equal(opt.state[p]["exp_avg"], opt2.state[q]["exp_avg"])
        p.grad = torch.full_like(p, 0.5)
        q.grad = torch.full_like(q, 0.5)
    opt.step()
    opt2.step()
    for p, q in zip(ps, ps2):
        assert torch.equal(p, q)


def _micro_model():
    from bench import build
    cfg = make_config()
    model, crit = build(cfg, DEV)
    return cfg, model, crit


def _batch(cfg):
    from retr_amd.synthetic import synthetic_captions, synthetic_images
    img, mask = synthetic_images(2, 64, seed=5)
    caps, cm = synthetic_captions(2, cfg.max_position_embeddings, cfg.vocab_size, seed=6)
    return (NestedTensor(img.to(DEV), mask.to(DEV)),), caps.to(DEV), cm.to(DEV)


def _groups(model, cfg):
    return [{"params": [p for n, p in model.named_parameters()
                        if "backbone" not in n and p.requires_grad]},
            {"params": [p for n, p in model.named_parameters()
                        if "backbone" in n and p.requires_grad], "lr": cfg.lr_backbone}]


@pytest.fixture
def deterministic_mode(request):
    from retr_amd import ops
    ops.set_deterministic(request.param)
    yield request.param
    ops.set_deterministic(False)


@pytest.mark.parametrize("deterministic_mode", [False, True], indirect=True)
def test_train_steps_fused_vs_torch_optimizer(deterministic_mode):
    """Three engine.train_step's with FusedAdamW (gradients written straight into the arena)
    against the same model with torch.optim.AdamW + clip_grad_norm_.  In deterministic mode
    both models' gradients come from identical fixed-order kernels, so only the optimizer
    arithmetic differs (2e-6 per step in test_fused_adamw_matches_torch, compounded over the
    three steps); otherwise split-K fp32 atomics add in a run-dependent order."""
    from retr_amd.engine import train_step
    tol_loss, tol_p = (1e-6, 1e-5) if deterministic_mode else (1e-5, 5e-5)
    cfg, m1, crit = _micro_model()
    _, m2, _ = _micro_model()
    o1 = FusedAdamW(_groups(m1, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    o2 = torch.optim.AdamW(_groups(m2, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay,
                           foreach=False)
    samples, caps, cm = _batch(cfg)
    m1.train()
    m2.train()
    for _ in range(3):
        l1 = train_step(m1, crit, samples, caps, cm, o1, 0.1)
        l2 = train_step(m2, crit, samples, caps, cm, o2, 0.1)
        assert abs(l1.item() - l2.item()) <= tol_loss * abs(l2.item())
    # gradients are written straight into the arena; only parameters with several
    # contributors (the learned query positions, shared by the decoder layers) are summed by
    # autograd outside it and copied in
    ps = [q for g in o1.param_groups for q in g["params"]]
    in_arena = sum(p.grad.data_ptr() == p._retr_grad_view.data_ptr() for p in ps)
    assert in_arena >= len(ps) - 2, (in_arena, len(ps))
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(a.detach(), b.detach()) < tol_p, n


@pytest.mark.parametrize("deterministic_mode", [False, True], indirect=True)
def test_gradient_accumulation_with_arena(deterministic_mode):
    """Two backward passes without zero_grad accumulate exactly like autograd's default
    (bitwise 2 g and g in deterministic mode)."""
    tol = 1e-7 if deterministic_mode else 1e-5     # fp32 atomics: order may differ
    cfg, model, crit = _micro_model()
    opt = FusedAdamW(_groups(model, cfg), lr=cfg.lr)
    samples, caps, cm = _batch(cfg)
    model.train()

    def loss():
        out = model(*samples, caps[:, :-1], cm[:, :-1])
        return crit(out.permute(0, 2, 1), caps[:, 1:])
    opt.zero_grad()
    loss().backward()
    g1 = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    loss().backward()
    for n, p in model.named_parameters():
        if n in g1:
            assert _rel(p.grad, 2 * g1[n]) < tol, n
    opt.zero_grad()
    loss().backward()
    for n, p in model.named_parameters():
        if n in g1:
            assert _rel(p.grad, g1[n]) < tol, n
            if deterministic_mode:
                assert torch.equal(p.grad, g1[n]), n


def test_graphed_step_with_fused_adamw_matches_eager():
    """engine.GraphedTrainStep (whole step in one hipGraph, FusedAdamW inside) against the same
    steps run eagerly: the gradient arena must be cleared on every replay."""
    from retr_amd.engine import GraphedTrainStep, train_step
    cfg, m1, crit = _micro_model()
    _, m2, _ = _micro_model()
    o1 = FusedAdamW(_groups(m1, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    o2 = FusedAdamW(_groups(m2, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    samples, caps, cm = _batch(cfg)
    m1.train()
    m2.train()
    graphed = GraphedTrainStep(m1, crit, o1, 0.1, warmup=2)
    # every call applies exactly one update (the warm-up steps are rolled back before capture)
    for _ in range(5):
        lg = graphed(samples, caps, cm).item()
    for _ in range(5):
        le = train_step(m2, crit, samples, caps, cm, o2, 0.1).item()
    assert abs(lg - le) <= 1e-5 * abs(le), (lg, le)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(a.detach(), b.detach()) < 5e-5, n


@pytest.mark.parametrize("deterministic_mode", [True], indirect=True)
def test_graphed_step_reads_its_own_input_buffers(deterministic_mode):
    """GraphedTrainStep.input_buffers(): a caller that writes the batch into the captured step's
    static inputs and passes them back gets the same updates as one passing its own tensors
    (which the step stages by a copy), including after the buffers are rewritten in place with
    a new batch."""
    from retr_amd.engine import GraphedTrainStep
    cfg, m1, crit = _micro_model()
    _, m2, _ = _micro_model()
    o1 = FusedAdamW(_groups(m1, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    o2 = FusedAdamW(_groups(m2, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    samples, caps, cm = _batch(cfg)
    m1.train()
    m2.train()
    g1 = GraphedTrainStep(m1, crit, o1, 0.1, warmup=2)
    g2 = GraphedTrainStep(m2, crit, o2, 0.1, warmup=2)
    l1 = [g1(samples, caps, cm).item()]
    l2 = [g2(samples, caps, cm).item()]
    st = g2.input_buffers()
    own = ((NestedTensor(st[0], st[1]),), st[2], st[3])
    for i in range(4):
        if i == 2:       # a new batch: the copy path stages it, the loader path writes in place
            samples = (NestedTensor(samples[0].tensors.flip(-1).contiguous(),
                                    samples[0].mask.clone()),)
            st[0].copy_(samples[0].tensors)
        l1.append(g1(samples, caps, cm).item())
        l2.append(g2(*own).item())
    assert l1 == l2, (l1, l2)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a.detach(), b.detach()), n


def test_graphed_and_eager_steps_mix_on_one_fused_adamw():
    """Consume mode (the captured update zeroes the gradient arena) belongs to GraphedTrainStep
    only: an eager train_step on the same optimizer between replays still leaves the clipped
    gradients in p.grad (torch semantics), and the next replay starts from a clean arena --
    same result as the same sequence of steps run eagerly."""
    from retr_amd.engine import GraphedTrainStep, train_step
    cfg, m1, crit = _micro_model()
    _, m2, _ = _micro_model()
    o1 = FusedAdamW(_groups(m1, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    o2 = FusedAdamW(_groups(m2, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    samples, caps, cm = _batch(cfg)
    m1.train()
    m2.train()
    graphed = GraphedTrainStep(m1, crit, o1, 0.1, warmup=2)
    assert o1.consume_grads is False
    graphed(samples, caps, cm)
    assert o1.consume_grads is False           # restored after warm-up + capture
    train_step(m1, crit, samples, caps, cm, o1, 0.1)
    g_eager = {n: p.grad.detach().clone() for n, p in m1.named_parameters()
               if p.grad is not None}
    assert g_eager and any(g.abs().max().item() > 0 for g in g_eager.values())
    lg = graphed(samples, caps, cm).item()
    for _ in range(3):
        le = train_step(m2, crit, samples, caps, cm, o2, 0.1).item()
    assert abs(lg - le) <= 1e-5 * abs(le), (lg, le)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(a.detach(), b.detach()) < 5e-5, n


def _micro_bf16(lr):
    from bench import build
    cfg = make_config(dtype="bf16")
    cfg.lr = lr
    model, crit = build(cfg, DEV)
    return cfg, model, crit


def _make_opt(kind, model, cfg):
    if kind == "fused":
        return FusedAdamW(_groups(model, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    return torch.optim.AdamW(_groups(model, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay,
                             capturable=True, foreach=False)


@pytest.mark.parametrize("kind", ["fused", "torch"])
def test_graphed_bf16_step_matches_eager_then_eval(kind):
    """The benchmarked path: GraphedTrainStep in bf16 (bf16 weight copies refreshed inside the
    replayed graph) == eager train_step, one update per call from the first call on; eager
    forwards and greedy decodes after replays see the replayed weights (no stale caches)."""
    from retr_amd.engine import GraphedTrainStep, train_step
    from retr_amd.eval_utils.decode import greedy
    lr = 2e-3                      # large enough that stale weights would be obvious
    cfg, m1, crit = _micro_bf16(lr)
    _, m2, _ = _micro_bf16(lr)
    o1, o2 = _make_opt(kind, m1, cfg), _make_opt(kind, m2, cfg)
    samples, caps, cm = _batch(cfg)
    graphed = GraphedTrainStep(m1, crit, o1, 0.1, warmup=2)

    def train(n):
        for _ in range(n):
            m1.train()
            m2.train()
            lg = graphed(samples, caps, cm).item()
            le = train_step(m2, crit, samples, caps, cm, o2, 0.1).item()
            assert abs(lg - le) <= 2e-3 * abs(le), (lg, le)

    def compare_eval():
        m1.eval()
        m2.eval()
        with torch.no_grad():
            a = m1(*samples, caps[:, :-1], cm[:, :-1]).float()
            b = m2(*samples, caps[:, :-1], cm[:, :-1]).float()
        assert ((a - b).norm() / b.norm()).item() < 1e-2
        ia = greedy(list(samples), m1, max_len=cfg.max_position_embeddings, bos_token=101,
                    eos_token=102)
        ib = greedy(list(samples), m2, max_len=cfg.max_position_embeddings, bos_token=101,
                    eos_token=102)
        assert (ia == ib).float().mean().item() > 0.9

    train(3)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(a.detach(), b.detach()) < 2e-3, n
    compare_eval()
    train(3)                     # replays after an eager eval (caches refreshed by the eval)
    compare_eval()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(a.detach(), b.detach()) < 2e-3, n
    if kind == "fused":
        s1, s2 = o1.state_dict(), o2.state_dict()
        for i in s2["state"]:
            assert float(s1["state"][i]["step"]) == float(s2["state"][i]["step"]) == 6.0


def test_fused_clip_nonfinite_norm_matches_torch():
    """A NaN gradient makes torch's clip coefficient NaN and every gradient NaN after
    clip_grad_norm_; the fused clip propagates it the same way."""
    ref = _params(3)
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    opt_r = torch.optim.AdamW(ref, lr=1e-3, foreach=False)
    opt_m = FusedAdamW([{"params": mine}], lr=1e-3)
    for pr, pm in zip(ref, mine):
        g = torch.ones_like(pr)
        pr.grad, pm.grad = g.clone(), g.clone()
    ref[1].grad[3] = float("nan")
    mine[1].grad[3] = float("nan")
    torch.nn.utils.clip_grad_norm_(ref, 0.1, foreach=False)
    opt_r.step()
    opt_m.step(max_norm=0.1)
    for pr, pm in zip(ref, mine):
        assert torch.isnan(pr.detach()).all() and torch.isnan(pm.detach()).all()
