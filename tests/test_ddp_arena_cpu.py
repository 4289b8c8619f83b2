"""Zero-copy data-parallel gradient sync on CPU (gloo, world_size 2): GradSync over an
optimizer gradient arena (the FusedAdamW layout: one flat fp32 ``G``, 64-byte aligned slots,
``p._retr_grad_view``; gradients written in place like the retr_amd backward kernels do) must
all-reduce in place, with buckets that are views of the arena, and give the gradients of the
concatenated batch; ``defer=True`` (graph-split steps) must give the same result."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Arena:
    """The attributes GradSync reads from retr_amd.optim.FusedAdamW."""

    def __init__(self, params):
        self._slots = {}
        off = 0
        for p in params:
            self._slots[id(p)] = (off, p.numel())
            off += (p.numel() + 15) // 16 * 16
        self.G = torch.zeros(off)
        for p in params:
            o, n = self._slots[id(p)]
            p._retr_grad_view = self.G[o:o + n].view_as(p)

    def covers(self, params):
        return all(id(p) in self._slots for p in params if p.requires_grad)


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 300), torch.nn.ReLU(),
                               torch.nn.Linear(300, 200), torch.nn.ReLU(),
                               torch.nn.Linear(200, 7))


def _loss(model, x, y):
    return torch.nn.functional.cross_entropy(model(x), y)


def _worker(rank, world, port, defer, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from retr_amd.ddp import GradSync
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 16, generator=g)
    y = torch.randint(0, 7, (8,), generator=g)
    ref_m = _model()
    _loss(ref_m, x, y).backward()
    ref = [p.grad.clone() for p in ref_m.parameters()]

    model = _model()
    params = list(model.parameters())
    arena = _Arena(params)
    sync = GradSync(params, bucket_mb=0.1, optimizer=arena, defer=defer)   # ~26k floats
    ok_views = sync.zero_copy and all(
        f.data_ptr() >= arena.G.data_ptr() and
        f.data_ptr() + 4 * f.numel() <= arena.G.data_ptr() + 4 * arena.G.numel()
        for f in sync.flat)
    # gradients land in the arena slots (what the retr_amd backward kernels do)
    for p in params:
        p.grad = p._retr_grad_view
    sl = slice(4 * rank, 4 * rank + 4)
    # a foreign gradient (not an arena view) for one parameter: copied in by the hook
    params[0].grad = torch.zeros_like(params[0])
    _loss(model, x[sl], y[sl]).backward()
    sync.synchronize()
    worst = max(((p.grad - r).norm() / r.norm().clamp_min(1e-12)).item()
                for p, r in zip(params, ref))
    in_arena = all(p.grad.data_ptr() == p._retr_grad_view.data_ptr() for p in params)
    q.put((rank, worst, len(sync.buckets), ok_views, in_arena))
    dist.destroy_process_group()


def _run(defer):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, defer, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, worst, nb, ok_views, in_arena in res:
        assert nb > 1, nb                       # several buckets
        assert ok_views                          # buckets are arena views (zero-copy)
        assert in_arena                          # averaged gradients live in the arena
        assert worst < 1e-6, (rank, worst)


def test_arena_gradsync_equals_concatenated_batch():
    _run(defer=False)


def test_arena_gradsync_deferred():
    _run(defer=True)
