"""Data-parallel engine behaviour on CPU (gloo, world_size 2):

* a non-finite loss on ONE rank stops EVERY rank with exit code 1 (engine.train_one_epoch agrees
  on the decision with one all-reduce; a lone exit would leave the peer blocked in the gradient
  all-reduce of that step -- reference engine.py:72-75 is single-process);
* with the zero-copy arena, a parameter that receives no gradient in step 2 gets zeros after the
  all-reduce, not step 1's averaged gradient (GradSync marks the arena dirty so its reset
  clears G);
* train_dp's validation loss is the reference's evaluate() over the exact validation set
  (SequentialSampler, main.py:52), computed on rank 0 and broadcast.
"""
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


def _spawn(fn, *args, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return res


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


class _TinyCaption(torch.nn.Module):
    """The Caption call signature (engine.py:70) on a toy body: logits [B, T, V]."""

    def __init__(self, V=11, C=8, poison=False):
        super().__init__()
        torch.manual_seed(0)
        self.emb = torch.nn.Embedding(V, C)
        self.img = torch.nn.Linear(3, C)
        self.out = torch.nn.Linear(C, V)
        self.poison = poison

    def forward(self, samples, caps, cap_mask):
        f = self.img(samples.tensors.mean(dim=(2, 3)))[:, None, :]
        z = self.out(torch.tanh(self.emb(caps) + f))
        return z * float("nan") if self.poison else z


class _Dataset(torch.utils.data.Dataset):
    return_global_context = False
    return_location_features = False

    def __init__(self, n, V=11, T=6, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.img = torch.randn(n, 3, 4, 4, generator=g)
        self.caps = torch.randint(1, V, (n, T + 1), generator=g)

    def __len__(self):
        return len(self.img)

    def __getitem__(self, i):
        return (i, self.img[i], torch.zeros(4, 4, dtype=torch.bool), self.caps[i],
                torch.zeros(self.caps.shape[1], dtype=torch.bool))


def _nan_worker(rank, world, port, q):
    _init(rank, world, port)
    from retr_amd.ddp import GradSync
    from retr_amd.engine import train_one_epoch
    model = _TinyCaption(poison=(rank == 1))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    sync = GradSync(list(model.parameters()), bucket_mb=1)
    loader = torch.utils.data.DataLoader(_Dataset(8, seed=rank), batch_size=2)
    code = None
    try:
        train_one_epoch(model, torch.nn.CrossEntropyLoss(), loader, opt, "cpu", 0, 0.1, sync)
    except SystemExit as e:
        code = e.code
    q.put((rank, code))
    dist.destroy_process_group()


def test_nonfinite_loss_on_one_rank_stops_all_ranks():
    res = _spawn(_nan_worker)
    assert res == [(0, 1), (1, 1)], res


class _ArenaOpt:
    """The FusedAdamW attributes GradSync reads, over a real retr_amd.optim._GradArena."""

    def __init__(self, params):
        from retr_amd.optim import _GradArena, _round
        self._slots, off = {}, 0
        for p in params:
            self._slots[id(p)] = (off, p.numel())
            off += _round(p.numel())
        self.G = torch.zeros(off)
        self.arena = _GradArena(self.G)
        for p in params:
            o, n = self._slots[id(p)]
            p._retr_grad_view = self.G[o:o + n].view_as(p)
            p._retr_arena = self.arena

    def covers(self, params):
        return all(id(p) in self._slots for p in params if p.requires_grad)

    def zero_grad(self, params):
        for p in params:
            p.grad = None
        self.arena.reset()


def _unused_worker(rank, world, port, q):
    _init(rank, world, port)
    from retr_amd.ddp import GradSync
    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(40))
    b = torch.nn.Parameter(torch.randn(24))
    params = [a, b]
    opt = _ArenaOpt(params)
    sync = GradSync(params, bucket_mb=1, optimizer=opt)
    # plain autograd: every gradient arrives outside the arena (no slot is handed out), the
    # case where nothing else marks G dirty
    opt.zero_grad(params)
    ((a * (rank + 1.0)).sum() + (b * (rank + 1.0)).sum()).backward()
    sync.synchronize()
    s1 = (a.grad.clone(), b.grad.clone())
    # step 2: b unused (its slot must read zero after the all-reduce, not step 1's average)
    opt.zero_grad(params)
    (a * (rank + 1.0)).sum().backward()
    sync.synchronize()
    q.put((rank, float(s1[0][0]), float(s1[1][0]), float(a.grad[0]), float(b.grad.abs().max())))
    dist.destroy_process_group()


def test_arena_unused_parameter_gets_zero_not_stale_gradient():
    res = _spawn(_unused_worker)
    for rank, a1, b1, a2, b2 in res:
        assert a1 == 1.5 and b1 == 1.5 and a2 == 1.5, (rank, a1, b1, a2)   # (1 + 2) / 2
        assert b2 == 0.0, (rank, b2)


def _val_worker(rank, world, port, q):
    _init(rank, world, port)
    from retr_amd.engine import evaluate
    from retr_amd.train_dp import _from_rank0, build_loaders

    class Cfg:
        batch_size, num_workers, seed = 3, 0, 42

    ds_val = _Dataset(7, seed=5)           # 7 = 3 + 3 + 1: a ragged last batch
    loader_train, loader_val, _ = build_loaders(Cfg, _Dataset(8), ds_val, rank, world)
    model = _TinyCaption()
    crit = torch.nn.CrossEntropyLoss()
    v = evaluate(model, crit, loader_val, "cpu") if loader_val is not None else None
    v = _from_rank0(v, "cpu", world)
    ref = evaluate(model, crit, torch.utils.data.DataLoader(ds_val, 3, shuffle=False), "cpu")
    q.put((rank, loader_val is not None, v, ref))
    dist.destroy_process_group()


def test_validation_loss_is_reference_evaluate_on_rank0():
    res = _spawn(_val_worker)
    assert [r[1] for r in res] == [True, False]
    for rank, _, v, ref in res:
        assert v == ref, (rank, v, ref)


def _schedule_worker(rank, world, port, q, mismatch):
    _init(rank, world, port)
    from retr_amd.ddp import check_schedule
    flat = [torch.zeros(64), torch.zeros(32), torch.zeros(16)]
    after = [[0], [], [1, 2]]
    if mismatch == "order" and rank == 1:
        after = [[0], [2], [1]]          # bucket 2 completed in another segment on rank 1
    if mismatch == "size" and rank == 1:
        flat[1] = torch.zeros(48)        # a bucket cut at other bounds
    try:
        sig = check_schedule(after, flat)
        q.put((rank, "ok", sig["after"]))
    except RuntimeError as e:
        q.put((rank, "raised", str(e)))
    dist.destroy_process_group()


def test_segmented_schedule_agreement_checked_across_ranks():
    """GraphedTrainStep pre-flight (ddp.check_schedule): every rank all-gathers its segment cut
    schedule + bucket sizes after capture; equal schedules pass, a rank whose hooks cut at
    another bucket or whose bucket bounds differ makes EVERY rank raise (no rank replays into
    a mismatched collective)."""
    ok = _spawn(_schedule_worker, None)
    assert [r[1] for r in ok] == ["ok", "ok"], ok
    assert ok[0][2] == [[0], [], [1, 2]]
    for mismatch in ("order", "size"):
        res = _spawn(_schedule_worker, mismatch)
        assert [r[1] for r in res] == ["raised", "raised"], (mismatch, res)
        assert "disagree" in res[0][2] and "rank 1" in res[0][2]
