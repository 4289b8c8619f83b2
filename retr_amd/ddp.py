"""Data-parallel gradient synchronisation for the RE⫶TR training step (new capability: the
reference is single-process).

One process per GPU; the global minibatch is sharded across ranks; after ``loss.backward()``
every trainable gradient is averaged over ranks with RCCL all-reduce (``torch.distributed``
backend "nccl" is RCCL on ROCm) so ``clip_grad_norm_`` and the optimizer see identical
gradients on every rank (== one process on the concatenated batch).

Buckets are filled in reverse registration order (≈ the order gradients become ready in
backward: head, decoder, encoder, backbone) from post-accumulate-grad hooks; a bucket's
all-reduce is launched asynchronously the moment its last gradient lands, so communication
overlaps the rest of the backward pass.  xGMI is point-to-point (7 links per GPU), so buckets
are large (default 64 MB) to amortise per-collective latency across RCCL's channels.
"""
import torch
import torch.distributed as dist


class GradSync:
    def __init__(self, params, bucket_mb=64, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params = [p for p in params if p.requires_grad]
        self.avg_supported = dist.get_backend(group) == "nccl"
        cap = int(bucket_mb * 2 ** 20) // 4
        self.buckets = []                     # list of lists of params
        cur, size = [], 0
        for p in reversed(self.params):
            if cur and size + p.numel() > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(cur)
        self.where = {}
        self.flat = []
        for bi, ps in enumerate(self.buckets):
            off = 0
            for p in ps:
                self.where[p] = (bi, off)
                off += p.numel()
            self.flat.append(torch.empty(off, dtype=torch.float32, device=ps[0].device))
        self.pending = [0] * len(self.buckets)
        self.handles = [None] * len(self.buckets)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self.reset()

    def reset(self):
        self.pending = [len(ps) for ps in self.buckets]
        self.handles = [None] * len(self.buckets)

    def _on_grad(self, p):
        bi, off = self.where[p]
        self.flat[bi][off:off + p.numel()].copy_(p.grad.reshape(-1))
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            op = dist.ReduceOp.AVG if self.avg_supported else dist.ReduceOp.SUM
            self.handles[bi] = dist.all_reduce(self.flat[bi], op=op, group=self.group,
                                               async_op=True)

    def synchronize(self):
        """Wait for every bucket (launching any whose gradients never arrived, e.g. unused
        parameters, with zeros) and write the averaged gradients back."""
        for bi, ps in enumerate(self.buckets):
            if self.handles[bi] is None:
                for p in ps:
                    if p.grad is None:
                        _, off = self.where[p]
                        self.flat[bi][off:off + p.numel()].zero_()
                op = dist.ReduceOp.AVG if self.avg_supported else dist.ReduceOp.SUM
                self.handles[bi] = dist.all_reduce(self.flat[bi], op=op, group=self.group,
                                                   async_op=True)
        for bi, ps in enumerate(self.buckets):
            self.handles[bi].wait()
            flat = self.flat[bi]
            if not self.avg_supported:
                flat.div_(self.world)
            for p in ps:
                _, off = self.where[p]
                g = flat[off:off + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
        self.reset()


def broadcast_parameters(module, src=0, group=None):
    """Rank-0 weights to all ranks (mirrors rank-0-only pretrained load, backbone.py:87-88)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t, src, group=group)
