"""Data-parallel gradient synchronisation for the RE⫶TR training step (new capability: the
reference is single-process; its loop is main.py:75-103 over a RandomSampler,
main.py:51-60).

One process per GPU; the global minibatch is sharded across ranks; after ``loss.backward()``
every trainable gradient is averaged over ranks with RCCL all-reduce (``torch.distributed``
backend "nccl" is RCCL on ROCm) so ``clip_grad_norm_`` and the optimizer see identical
gradients on every rank (== one process on the concatenated batch).

Buckets.  With a ``FusedAdamW`` that manages every parameter, the buckets ARE contiguous ranges
of its fp32 gradient arena ``G`` (the backward kernels already write there): a bucket's
all-reduce runs in place on the arena view, with no copy in or out (zero-copy).  Buckets are
cut from the end of the arena backwards (head and decoder first, ≈ the order gradients become
ready in backward).  Any other optimizer gets flat fp32 bucket buffers that gradients are
copied into and back out of.  xGMI is point-to-point (7 links per GPU): buckets are large
(default 64 MB) to amortise per-collective latency across RCCL's channels.

Overlap.  In eager steps each bucket's all-reduce is launched asynchronously from a
post-accumulate-grad hook the moment its last gradient lands, overlapping the rest of
backward.  ``defer=True`` (hipGraph-captured steps, engine.GraphedTrainStep): the hooks only
route gradients into the buckets; ``synchronize()`` launches every bucket's all-reduce between
the captured forward/backward graph and the captured optimizer graph.
"""
import torch
import torch.distributed as dist

from .optim import _round


class GradSync:
    def __init__(self, params, bucket_mb=64, group=None, optimizer=None, defer=False):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params = [p for p in params if p.requires_grad]
        self.avg_supported = dist.get_backend(group) == "nccl"
        self.defer = defer
        cap = int(bucket_mb * 2 ** 20) // 4
        self.arena = self._arena_of(optimizer)
        self.buckets = []                     # list of lists of params
        self.flat = []                        # fp32 bucket tensors (arena views or buffers)
        self.where = {}
        if self.arena is not None:
            opt = self.arena
            slots = sorted(((opt._slots[id(p)][0], p) for p in self.params), key=lambda t: -t[0])
            cur, lo, hi = [], None, None
            for off, p in slots:
                end = off + _round(p.numel())
                if cur and hi - off > cap:
                    self._add_arena_bucket(cur, lo, hi)
                    cur, hi = [], None
                if hi is None:
                    hi = end
                lo = off
                cur.append(p)
            if cur:
                self._add_arena_bucket(cur, lo, hi)
        else:
            cur, size = [], 0
            for p in reversed(self.params):
                if cur and size + p.numel() > cap:
                    self.buckets.append(cur)
                    cur, size = [], 0
                cur.append(p)
                size += p.numel()
            if cur:
                self.buckets.append(cur)
            for bi, ps in enumerate(self.buckets):
                off = 0
                for p in ps:
                    self.where[p] = (bi, off)
                    off += p.numel()
                self.flat.append(torch.empty(off, dtype=torch.float32, device=ps[0].device))
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)
        self.foreign = set()
        self.on_ready = None                  # deferred mode: callback(bucket) at completion
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self.reset()

    def _arena_of(self, optimizer):
        """The optimizer's gradient arena (retr_amd.optim.FusedAdamW: ``G``, ``_slots``,
        ``covers``; every parameter carries ``_retr_grad_view``) if it manages all params."""
        if (optimizer is not None and getattr(optimizer, "G", None) is not None
                and hasattr(optimizer, "_slots") and optimizer.covers(self.params)
                and all(hasattr(p, "_retr_grad_view") for p in self.params)):
            return optimizer
        return None

    def _add_arena_bucket(self, ps, lo, hi):
        bi = len(self.buckets)
        self.buckets.append(ps)
        for p in ps:
            self.where[p] = (bi, self.arena._slots[id(p)][0] - lo)
        self.flat.append(self.arena.G[lo:hi])

    @property
    def zero_copy(self):
        return self.arena is not None

    def _mark_dirty(self):
        """G now holds values the optimizer's arena bookkeeping did not hand out (a copied-in
        gradient, or the all-reduce's in-place result): make its next reset zero G."""
        a = getattr(self.arena, "arena", None)
        if a is not None:
            a.dirty = True

    def all_finite(self, finite):
        """True iff ``finite`` holds on every rank (one MAX all-reduce of a flag)."""
        dev = self.params[0].device if self.params else torch.device("cpu")
        if self.avg_supported and dev.type != "cuda":
            dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([0.0 if finite else 1.0], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.item() == 0.0

    def reset(self):
        self.pending = [len(ps) for ps in self.buckets]
        self.handles = [None] * len(self.buckets)

    def _op(self):
        return dist.ReduceOp.AVG if self.avg_supported else dist.ReduceOp.SUM

    def _launch(self, bi):
        self.handles[bi] = dist.all_reduce(self.flat[bi], op=self._op(), group=self.group,
                                           async_op=True)

    def _on_grad(self, p):
        bi, off = self.where[p]
        from . import ops
        if self.arena is not None:
            view = p._retr_grad_view
            if p.grad.data_ptr() != view.data_ptr():     # produced outside the arena
                ops.flush_wgrad()
                view.copy_(p.grad)
                self.foreign.add(p)
                self._mark_dirty()
        else:
            ops.flush_wgrad()
            self.flat[bi][off:off + p.numel()].copy_(p.grad.reshape(-1))
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            # the bucket's gradients may still sit in the deferred weight-gradient queue
            ops.flush_wgrad()
            if not self.defer:
                self._launch(bi)
            elif self.on_ready is not None:
                self.on_ready(bi)

    def check_schedule(self, after):
        """``check_schedule`` over this GradSync's buckets and group (see there)."""
        return check_schedule(after, self.flat, self.group)

    def synchronize(self):
        """Wait for every bucket (launching the ones not launched yet: deferred mode, or
        parameters that received no gradient, whose slots hold zeros) and leave the averaged
        gradients in ``p.grad``."""
        for bi, ps in enumerate(self.buckets):
            if self.handles[bi] is None:
                if self.arena is None:
                    for p in ps:
                        if p.grad is None:
                            _, off = self.where[p]
                            self.flat[bi][off:off + p.numel()].zero_()
                self._launch(bi)
        for bi, ps in enumerate(self.buckets):
            self.handles[bi].wait()
            flat = self.flat[bi]
            if not self.avg_supported:
                flat.div_(self.world)
            if self.arena is not None:
                self._mark_dirty()
                for p in ps:
                    if p.grad is None or p in self.foreign:
                        p.grad = p._retr_grad_view.view(p.shape)
                continue
            for p in ps:
                _, off = self.where[p]
                g = flat[off:off + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
        self.foreign.clear()
        self.reset()


def schedule_signature(after, flat):
    """What every rank must agree on before replaying a segmented DP step: the buckets whose
    all-reduce follows each segment (``GraphedTrainStep.after``) and every bucket's element
    count.  Plain ints only, so the signature compares exactly across processes."""
    return {"after": [[int(b) for b in a] for a in after],
            "bucket_numel": [int(f.numel()) for f in flat]}


def check_schedule(after, flat, group=None):
    """Pre-flight for the segmented, hipGraph-replayed DP step (engine.GraphedTrainStep).

    Each rank derives its segment cuts from its OWN autograd hook order at capture time.  If two
    ranks ever cut differently (different bucket order, a bucket completing in another segment,
    different bucket sizes), their replays would enqueue mismatched RCCL all-reduces and hang
    or average the wrong bytes.  All-gather every rank's ``schedule_signature`` and raise on
    any difference -- once, after capture, before the first replay.  Returns the signature."""
    mine = schedule_signature(after, flat)
    world = dist.get_world_size(group)
    if world == 1:
        return mine
    got = [None] * world
    dist.all_gather_object(got, mine, group=group)
    bad = [r for r, sig in enumerate(got) if sig != got[0]]
    if bad:
        rows = "; ".join(f"rank {r}: after={got[r]['after']} "
                         f"buckets={got[r]['bucket_numel']}" for r in [0] + bad)
        raise RuntimeError("GradSync: ranks disagree on the segmented all-reduce schedule "
                           f"(ranks {bad} differ from rank 0): {rows}")
    return mine


def broadcast_parameters(module, src=0, group=None):
    """Rank-0 weights to all ranks (mirrors rank-0-only pretrained load, backbone.py:87-88)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t, src, group=group)
