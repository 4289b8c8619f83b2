"""Fused gradient clipping + AdamW over flat parameter / gradient arenas (MI355X).

Drop-in for the reference's optimizer step (main.py:39-41 builds ``torch.optim.AdamW`` over two
param groups; engine.py:80-83 runs ``clip_grad_norm_`` then ``optimizer.step()``):

    optimizer = FusedAdamW(param_dicts, lr=config.lr, weight_decay=config.weight_decay)
    ...
    optimizer.step(max_norm=max_norm)      # == clip_grad_norm_(params, max_norm); step()

Layout.  At construction every parameter of every group is moved into one fp32 arena ``P``
(group after group, each parameter 64-byte aligned; ``p.data`` becomes a view), with matching
arenas ``G`` (gradients), ``M`` / ``V`` (moments).  The HIP kernels (retr_amd/csrc/optim.hip)
then update a whole group in one streaming pass.  The gradient arena is also where the
backward kernels write: ``grad_slot(p)`` (used by every retr_amd autograd Function) hands out
the zeroed ``G`` view of a parameter the first time it receives a gradient after a reset, so
AccumulateGrad adopts it without a copy and no per-parameter zero-fill is needed.  Gradients
that arrive elsewhere (a second contributor, a non-retr op, user code) are copied in before
the update, so results never depend on who produced them.

Semantics match torch.optim.AdamW (amsgrad=False, maximize=False) + clip_grad_norm_ up to
fp32 rounding; parameters whose ``.grad`` is None are skipped (no decay, no moment update).
The step counter and the hyper-parameters (lr, weight_decay per group) live on the device so
a hipGraph-captured step replays correctly; ``sync_hyper()`` pushes host-side lr changes
(e.g. from a StepLR scheduler) before a replay.
"""
import torch

from ._lib import call, ptr, stream

_ALIGN = 16          # floats per arena slot alignment (64 B)
_NPARTS = 512        # norm partials per contiguous segment


def _round(n, a=_ALIGN):
    return (n + a - 1) // a * a


class _GradArena:
    """Bookkeeping for handing out zeroed gradient views (see module docstring)."""

    def __init__(self, G):
        self.G = G
        self.handed = set()
        self.dirty = False

    def hand_out(self, p):
        if p.grad is not None or id(p) in self.handed:
            return None
        self.handed.add(id(p))
        self.dirty = True
        # a new view object: AccumulateGrad adopts a returned gradient only when nothing else
        # references its TensorImpl (``p._retr_grad_view`` itself would force a copy)
        return p._retr_grad_view.view(p.shape)

    def reset(self):
        if self.dirty:
            self.G.zero_()
        self.handed.clear()
        self.dirty = False


def grad_slot(p):
    """Zeroed fp32 gradient buffer for parameter ``p`` to accumulate into and return from an
    autograd Function, or None (caller allocates a zeroed buffer of its own)."""
    a = getattr(p, "_retr_arena", None)
    if a is None:
        return None
    return a.hand_out(p)


# Called with ``p`` when a parameter whose arena slot was already handed out this pass gets a
# second gradient contributor (ops sets it: flushes deferred sums aimed at that slot, because
# autograd is about to read the slot to add the two contributions).
REUSE_HOOK = None


def grad_buffer(p, shape=None):
    """(buffer, from_arena): a zeroed fp32 buffer shaped like ``p`` (or ``shape``)."""
    v = grad_slot(p)
    if v is not None:
        return (v if shape is None else v.view(shape)), True
    a = getattr(p, "_retr_arena", None)
    if a is not None and REUSE_HOOK is not None and id(p) in a.handed:
        REUSE_HOOK(p)
    return torch.zeros(shape if shape is not None else p.shape, dtype=torch.float32,
                       device=p.device), False


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 amsgrad=False, maximize=False, bf16_shadow=True, **unused):
        if amsgrad or maximize:
            raise NotImplementedError("FusedAdamW: amsgrad / maximize are not supported")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=True, differentiable=False,
                        fused=None)
        super().__init__(params, defaults)
        self._shadow = bool(bf16_shadow)
        self._build()

    # -- arena construction ----------------------------------------------------------------
    def _build(self):
        plist = [p for g in self.param_groups for p in g["params"]]
        if len({id(p) for p in plist}) != len(plist):
            raise ValueError("FusedAdamW: a parameter appears in more than one group")
        dev = plist[0].device
        for p in plist:
            if p.dtype != torch.float32 or not p.is_cuda or p.is_sparse:
                raise TypeError("FusedAdamW: fp32 dense device parameters only")
            if p.device != dev:
                raise ValueError("FusedAdamW: all parameters must be on one device")
        self._slots = {}
        self._groups = []         # (lo, hi) element range of each group
        off = 0
        for g in self.param_groups:
            lo = off
            for p in g["params"]:
                self._slots[id(p)] = (off, p.numel())
                off += _round(max(p.numel(), self._padded_numel(p)))
            self._groups.append((lo, off))
        total = max(off, _ALIGN)
        self.P = torch.zeros(total, dtype=torch.float32, device=dev)
        self.G = torch.zeros_like(self.P)
        self.M = torch.zeros_like(self.P)
        self.V = torch.zeros_like(self.P)
        # bf16 shadow of P, rewritten by every update: the compute-dtype weight copies the GEMMs
        # read (ops._WeightCache hands out p._retr_shadow while it is current)
        self.P16 = torch.empty(total, dtype=torch.bfloat16, device=dev) if self._shadow else None
        self.arena = _GradArena(self.G)
        # consume mode (set by engine.GraphedTrainStep): the update zeroes the stepped gradient
        # ranges instead of writing the clipped gradients back, so the next step needs no zero
        # fill of the arena; p.grad then reads zero after step()
        self.consume_grads = False
        self._step_t = torch.zeros(1, dtype=torch.float32, device=dev)   # device step count
        self._global = 0                                  # host mirror of _step_t
        self._counts = {id(p): 0 for p in plist}          # per-parameter step (torch semantics)
        self._hyper = torch.zeros(len(self.param_groups), 2, dtype=torch.float32, device=dev)
        self._hyper_host = None
        self._partials = torch.zeros(_NPARTS * 2 * len(self.param_groups) + _NPARTS,
                                     dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p in plist:
                o, n = self._slots[id(p)]
                view = self.P[o:o + n].view_as(p)
                view.copy_(p.data)
                p.data = view
                p._retr_grad_view = self.G[o:o + n].view_as(p)
                p._retr_arena = self.arena
                if self.P16 is not None:
                    p._retr_shadow = self.P16[o:o + n].view_as(p)
                pn = self._padded_numel(p)
                if pn > n:   # rows past the parameter: never written, so always zero
                    shape = (p._retr_pad_rows,) + tuple(p.shape[1:])
                    p._retr_pad_data = self.P[o:o + pn].view(shape)
                    if self.P16 is not None:
                        p._retr_pad_shadow = self.P16[o:o + pn].view(shape)
                self.state[p] = {"exp_avg": self.M[o:o + n].view_as(p),
                                 "exp_avg_sq": self.V[o:o + n].view_as(p)}
        self.sync_hyper()
        self.sync_shadow()

    @staticmethod
    def _padded_numel(p):
        """Elements of ``p`` zero-padded to ``p._retr_pad_rows`` rows (models/caption.py MLP):
        the slot reserves them so padded views of P / P16 need no copies."""
        rows = getattr(p, "_retr_pad_rows", 0)
        return rows * (p.numel() // p.shape[0]) if rows > p.shape[0] else 0

    def sync_shadow(self):
        """Re-cast the whole bf16 shadow from P (after P was written outside step())."""
        if self.P16 is None:
            return
        call("retr_cast", 1, ptr(self.P), ptr(self.P16), self.P.numel(), stream())
        self.mark_shadow_fresh([p for g in self.param_groups for p in g["params"]])

    def mark_shadow_fresh(self, params):
        """Record that the shadow of ``params`` holds their current values (their autograd
        version as of now): ops._WeightCache then serves it without a cast."""
        if self.P16 is None:
            return
        for p in params:
            p._retr_shadow_ver = (p._version, p.data_ptr())

    def sync_hyper(self):
        """Copy (lr, weight_decay) of every group to the device if they changed."""
        h = [(float(g["lr"]), float(g["weight_decay"])) for g in self.param_groups]
        if h != self._hyper_host:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedAdamW: hyper-parameters changed during graph capture")
            self._hyper.copy_(torch.tensor(h, dtype=torch.float32))
            self._hyper_host = h

    def covers(self, params):
        """True if every parameter in ``params`` that requires grad is managed here."""
        return all(id(p) in self._slots for p in params if p.requires_grad)

    # -- optimizer API ---------------------------------------------------------------------
    def zero_grad(self, set_to_none=True):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                if set_to_none:
                    p.grad = None
                elif p.grad.data_ptr() != p._retr_grad_view.data_ptr():
                    p.grad.zero_()
        if torch.cuda.is_current_stream_capturing() and not self.consume_grads:
            # a captured step must clear G on every replay, whatever the host-side dirty flag
            # says at capture time (the memset before capture leaves it False); in consume mode
            # every replay's update leaves G zero instead
            self.arena.dirty = True
        self.arena.reset()
        if not set_to_none:
            # gradients stay allocated (views of G or foreign tensors) and autograd adds into
            # them: never hand out slots, and zero G again at the next reset
            self.arena.handed.update(id(p) for g in self.param_groups for p in g["params"])
            self.arena.dirty = True

    def _segments(self):
        """Maximal runs of consecutive parameters (within one group, same step count) that
        have gradients; gradients living outside the arena are copied in."""
        segs, foreign, active = [], [], []
        for gi, g in enumerate(self.param_groups):
            run = None
            for p in g["params"]:
                o, n = self._slots[id(p)]
                off = self._counts[id(p)] - self._global
                if p.grad is None or (run is not None and run[3] != off):
                    if run is not None:
                        segs.append(run)
                        run = None
                    if p.grad is None:
                        continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdamW does not support sparse gradients")
                if p.grad.data_ptr() != p._retr_grad_view.data_ptr():
                    p._retr_grad_view.copy_(p.grad)
                    foreign.append(p)
                    self.arena.dirty = True
                active.append(p)
                if run is None:
                    run = [gi, o, o + _round(n), off]
                else:
                    run[2] = o + _round(n)
            if run is not None:
                segs.append(run)
        return segs, foreign, active

    @torch.no_grad()
    def step(self, closure=None, max_norm=0.0):
        """AdamW step; with ``max_norm > 0`` first clip the global gradient 2-norm (exactly
        ``torch.nn.utils.clip_grad_norm_(params, max_norm)`` over this optimizer's params)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not torch.cuda.is_current_stream_capturing():
            self.sync_hyper()
        segs, foreign, active = self._segments()
        if not segs:
            return loss
        nparts = _NPARTS * len(segs)
        if nparts > self._partials.numel():
            self._partials = torch.zeros(nparts, dtype=torch.float32, device=self.P.device)
        st = stream()
        clip = float(max_norm) > 0
        for k, (gi, lo, hi, _) in enumerate(segs):
            call("retr_adamw_sumsq", ptr(self.G) + 4 * lo if clip else None, hi - lo,
                 ptr(self._partials) + 4 * _NPARTS * k, _NPARTS,
                 ptr(self._step_t) if k == 0 else None, st)
        b1, b2 = self.param_groups[0]["betas"]
        eps = self.param_groups[0]["eps"]
        for gi, lo, hi, off in segs:
            g = self.param_groups[gi]
            if tuple(g["betas"]) != (b1, b2) or g["eps"] != eps:
                b1, b2 = g["betas"]
                eps = g["eps"]
            call("retr_adamw_update2", ptr(self.P) + 4 * lo, ptr(self.G) + 4 * lo,
                 ptr(self.M) + 4 * lo, ptr(self.V) + 4 * lo, hi - lo, ptr(self._hyper) + 8 * gi,
                 float(b1), float(b2), float(eps), ptr(self._step_t), float(off),
                 ptr(self._partials), nparts, float(max_norm) if clip else 0.0,
                 ptr(self.P16) + 2 * lo if self.P16 is not None else None,
                 int(self.consume_grads), st)
        self._advance_host(active)
        self._last_active = active
        if self.consume_grads:
            # the update zeroed G over every stepped range; the arena is clean for the next
            # step unless a handed-out slot belongs to a parameter that was not stepped
            stepped = {id(p) for p in active}
            if self.arena.handed <= stepped:
                self.arena.dirty = False
        else:
            for p in foreign:      # clipped values back into gradients living elsewhere
                if clip:
                    p.grad.copy_(p._retr_grad_view)
        _bump_versions(self.param_groups)
        self.mark_shadow_fresh(active)     # the update wrote their shadow too
        return loss

    def _advance_host(self, active):
        """Host mirror of one executed step (called by step(), and by GraphedTrainStep after
        every replay of a captured step, whose kernels advance only the device counter)."""
        self._global += 1
        for p in active:
            self._counts[id(p)] += 1

    def snapshot(self):
        """Device copies of parameters / moments / step counter plus the host counters."""
        return (self.P.clone(), self.M.clone(), self.V.clone(), self._step_t.clone(),
                self._global, dict(self._counts))

    def restore(self, snap):
        """In-place restore of ``snapshot()`` (pointers stay valid for captured graphs)."""
        P, M, V, t, g, counts = snap
        with torch.no_grad():
            self.P.copy_(P)
            self.M.copy_(M)
            self.V.copy_(V)
            self._step_t.copy_(t)
        self._global = g
        self._counts = dict(counts)
        self.sync_shadow()

    def state_dict(self):
        """torch.optim.AdamW layout: per-parameter 'step' (CPU float tensor) + moments."""
        sd = super().state_dict()
        idx = [i for g in sd["param_groups"] for i in g["params"]]
        plist = [p for g in self.param_groups for p in g["params"]]
        for i, p in zip(idx, plist):
            st = dict(sd["state"].get(i, {}))
            st["step"] = torch.tensor(float(self._counts[id(p)]))
            sd["state"][i] = st
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        # re-seat the loaded moments into the arenas; step counts back to host + device
        with torch.no_grad():
            for g in self.param_groups:
                for p in g["params"]:
                    o, n = self._slots[id(p)]
                    s = self.state.get(p, {})
                    m, v = self.M[o:o + n].view_as(p), self.V[o:o + n].view_as(p)
                    if "exp_avg" in s:
                        m.copy_(s["exp_avg"])
                        v.copy_(s["exp_avg_sq"])
                    self._counts[id(p)] = int(float(s["step"])) if "step" in s else 0
                    self.state[p] = {"exp_avg": m, "exp_avg_sq": v}
            self._global = max(self._counts.values(), default=0)
            self._step_t.fill_(float(self._global))
        self._hyper_host = None
        self.sync_hyper()


def _bump_versions(groups):
    """The kernels write parameters through raw pointers; tell autograd / the compute-copy
    caches (ops._WeightCache keys on ``_version``) that they changed."""
    inc = torch.autograd.graph.increment_version
    for g in groups:
        for p in g["params"]:
            if p.grad is not None:
                inc(p)
