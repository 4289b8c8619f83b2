"""The RCCL data-parallel path on the GPU: a world_size-1 process group over the ``nccl``
backend (RCCL on ROCm), so every all-reduce really executes on the device.  GradSync on the
retr_amd model with FusedAdamW (zero-copy buckets on the gradient arena), the graph-split
captured step with the all-reduce between the two graphs, and the torchrun-style launcher
(retr_amd.train_dp, DistributedSampler; reference main.py:51-60, 75-103)."""
import math
import socket

import pytest
import torch
import torch.distributed as dist

from retr_amd.models.utils import NestedTensor
from tests.helpers import make_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def pg():
    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                                world_size=1)
        created = True
    yield
    if created:
        dist.destroy_process_group()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def _setup(dtype):
    from bench import build, make_optimizer
    from retr_amd.synthetic import synthetic_captions, synthetic_images
    cfg = make_config(dtype=dtype)
    m1, crit = build(cfg, DEV)
    m2, _ = build(cfg, DEV)
    o1 = make_optimizer(m1, cfg, fused=True)
    o2 = make_optimizer(m2, cfg, fused=True)
    img, mask = synthetic_images(2, 64, seed=5, pad_band=True)
    caps, cm = synthetic_captions(2, cfg.max_position_embeddings, cfg.vocab_size, seed=6)
    samples = (NestedTensor(img.to(DEV), mask.to(DEV)),)
    m1.train()
    m2.train()
    return cfg, m1, m2, o1, o2, crit, samples, caps.to(DEV), cm.to(DEV)


def _counting(gs):
    gs.launches = 0
    orig = gs._launch

    def launch(bi):
        gs.launches += 1
        orig(bi)
    gs._launch = launch
    return gs


def test_gradsync_zero_copy_rccl(pg):
    from retr_amd.ddp import GradSync
    from retr_amd.engine import train_step
    cfg, m1, m2, o1, o2, crit, samples, caps, cm = _setup("bf16")
    gs = _counting(GradSync([p for p in m1.parameters() if p.requires_grad], bucket_mb=2,
                            optimizer=o1))
    assert gs.zero_copy and gs.avg_supported and len(gs.buckets) > 1
    lo, hi = o1.G.data_ptr(), o1.G.data_ptr() + 4 * o1.G.numel()
    assert all(lo <= f.data_ptr() and f.data_ptr() + 4 * f.numel() <= hi for f in gs.flat)
    for _ in range(3):
        l1 = train_step(m1, crit, samples, caps, cm, o1, cfg.clip_max_norm, gs)
        l2 = train_step(m2, crit, samples, caps, cm, o2, cfg.clip_max_norm)
        assert abs(l1.item() - l2.item()) <= 1e-6 * abs(l2.item())
    assert gs.launches == 3 * len(gs.buckets)          # every bucket all-reduced every step
    ps = [p for g in o1.param_groups for p in g["params"]]
    assert all(p.grad.data_ptr() == p._retr_grad_view.data_ptr() for p in ps)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(a.detach(), b.detach()) < 1e-6, n


def test_graphed_step_with_gradsync_rccl(pg):
    """GraphedTrainStep with a GradSync: forward/backward graph, RCCL all-reduce, optimizer
    graph -- equal to the same steps run eagerly without data parallelism."""
    from retr_amd.ddp import GradSync
    from retr_amd.engine import GraphedTrainStep, train_step
    cfg, m1, m2, o1, o2, crit, samples, caps, cm = _setup("bf16")
    gs = _counting(GradSync([p for p in m1.parameters() if p.requires_grad], bucket_mb=2,
                            optimizer=o1))
    step = GraphedTrainStep(m1, crit, o1, cfg.clip_max_norm, grad_sync=gs)
    for _ in range(3):
        l1 = step(samples, caps, cm)
        l2 = train_step(m2, crit, samples, caps, cm, o2, cfg.clip_max_norm)
        assert abs(l1.item() - l2.item()) <= 1e-5 * abs(l2.item())
    assert step.graph_opt is not None
    assert gs.launches >= 3 * len(gs.buckets)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(a.detach(), b.detach()) < 1e-5, n


def test_train_dp_launcher(pg, tmp_path):
    from retr_amd.synthetic import SyntheticRefDataset
    from retr_amd.train_dp import main
    cfg = make_config()
    cfg.batch_size, cfg.num_workers, cfg.device = 2, 0, DEV
    hist = main(cfg, SyntheticRefDataset(cfg, 6, 64), SyntheticRefDataset(cfg, 4, 64, seed=3),
                epochs=2, checkpoint_dir=str(tmp_path))
    assert [h[0] for h in hist] == [0, 1]
    assert all(math.isfinite(h[1]) and math.isfinite(h[2]) for h in hist)
    ck = torch.load(tmp_path / f"{cfg.transformer_type}_{cfg.prefix}_checkpoint_1.pth",
                    map_location="cpu", weights_only=True)
    assert ck["epoch"] == 1 and "model_state_dict" in ck and "optimizer_state_dict" in ck


def test_segmented_dp_step_cfg2_equals_single_graph_bitwise(pg):
    """bench.py's N>1 objects at the full cfg2 shape (R50 6/6 d256, 640x640, batch 16, bf16,
    dropout 0.1, FusedAdamW, GradSync with the bench's 64 MB buckets): the segmented capture
    (forward/backward cut at bucket completions, each bucket's RCCL all-reduce enqueued
    right after the segment it completed in) gives bitwise the same losses and weights as the
    single-graph non-DP step (world 1: AVG over one rank is the identity).  Deterministic
    reductions on both sides so the comparison can be bitwise."""
    from bench import build, cfg2, make_optimizer
    from retr_amd import ops
    from retr_amd.ddp import GradSync
    from retr_amd.engine import GraphedTrainStep
    from retr_amd.synthetic import synthetic_captions, synthetic_images
    cfg = cfg2()
    cfg.deterministic = True
    try:
        m1, crit = build(cfg, DEV)
        m2, _ = build(cfg, DEV)
        o1 = make_optimizer(m1, cfg, capturable=True, fused=True)
        o2 = make_optimizer(m2, cfg, capturable=True, fused=True)
        gs = GradSync([p for p in m1.parameters() if p.requires_grad],
                      bucket_mb=cfg.grad_bucket_mb, optimizer=o1)
        s1 = GraphedTrainStep(m1, crit, o1, cfg.clip_max_norm, gs)
        s2 = GraphedTrainStep(m2, crit, o2, cfg.clip_max_norm)
        img, mask = synthetic_images(16, 640, seed=1000)
        caps, cm = synthetic_captions(16, cfg.max_position_embeddings, cfg.vocab_size, seed=2000)
        samples = (NestedTensor(img.to(DEV), mask.to(DEV)),)
        caps, cm = caps.to(DEV), cm.to(DEV)
        m1.train()
        m2.train()
        for _ in range(3):
            # the same dropout streams on both sides: device step seed and host per-op counter
            seed, ctr = ops.seed_base().clone(), ops._seed_state["ctr"]
            l1 = s1(samples, caps, cm).clone()
            ops.seed_base().copy_(seed)
            ops._seed_state["ctr"] = ctr
            l2 = s2(samples, caps, cm).clone()
            torch.cuda.synchronize()
            assert torch.isfinite(l1).all()
            assert torch.equal(l1, l2), (l1.item(), l2.item())
        assert torch.equal(o1.P, o2.P)
        assert torch.equal(o1.M, o2.M) and torch.equal(o1.V, o2.V)
        # the schedule: several segments, every bucket all-reduced exactly once, each right
        # after the segment it completed in and before the next segment's replay
        nb = len(gs.buckets)
        assert nb >= 3 and len(s1.segments) >= 2
        seen = [b for kind, b in s1.order if kind == "allreduce"]
        assert sorted(seen) == list(range(nb)), s1.order
        for i, (kind, v) in enumerate(s1.order):
            if kind == "allreduce":
                k = max(j for j in range(i) if s1.order[j][0] == "segment")
                assert v in s1.after[s1.order[k][1]]
        # overlap exists: at least one all-reduce is enqueued before the last segment's replay
        last = max(i for i, (kind, _) in enumerate(s1.order) if kind == "segment")
        assert any(kind == "allreduce" for kind, _ in s1.order[:last]), s1.order
    finally:
        ops.set_deterministic(False)
