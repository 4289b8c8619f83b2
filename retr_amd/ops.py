"""Autograd operators of the RE⫶TR hot path, each a thin host wrapper over libretr_hip.so.

Granularity follows the reference's residual sub-layers so the backward can fuse what the
reference computes as separate PyTorch ops:

* ``ln_pos``          LayerNorm (+ position add)         transformer_modules.py:31-34,58-62,89
* ``self_attn_block`` in-proj -> attention -> out-proj -> dropout -> residual   (:22-46)
* ``cross_attn_block``                                                           (:49-74)
* ``ffn_block``       Linear -> ReLU -> Linear -> dropout -> residual            (:6-11,77-97)
* ``embed_ln``        DecoderEmbeddings                                          (:100-129)
* ``linear``          input_proj (1x1 conv) and plain linears
* ``mlp_head``        MLP(C, 512, V, 3)                          models/caption.py:161-174
* ``cross_entropy``   CrossEntropyLoss (mean, no ignore_index)  caption.py:210 / engine.py:71
* ``backbone``        ResNet body (NHWC implicit-GEMM convs, FrozenBN folded) backbone.py:41-77

Tensors of the residual stream are fp32; GEMM operands are the compute dtype (bf16 or fp32).
All ops raise on non-HIP tensors (no CPU fallback).
"""
import ctypes
import os

import torch

from . import _lib
from . import optim as _optim
from .optim import grad_buffer
from ._lib import BF16, F32, call, ptr

# ---------------------------------------------------------------------------------------------
# runtime helpers
# ---------------------------------------------------------------------------------------------

_seed_state = {"base": None, "ctr": 0}


def next_seed():
    """Per-op dropout seed: a pure function of torch's initial seed and a call counter."""
    if _seed_state["base"] is None:
        _seed_state["base"] = torch.initial_seed() & 0xFFFFFFFFFFFF
    _seed_state["ctr"] += 1
    return (_seed_state["base"] * 0x100000001B3 + _seed_state["ctr"] * 0x9E3779B1) & (2**63 - 1)


_seed_base = {}


def seed_base(device=None):
    """Device-resident step seed shared by every dropout mask (see retr_set_seed_base)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    t = _seed_base.get(dev)
    if t is None:
        t = torch.full((1,), (torch.initial_seed() * 0x9E3779B97F4A7C15) & (2 ** 62 - 1),
                       dtype=torch.int64, device=dev)
        _seed_base[dev] = t
        call("retr_set_seed_base", ptr(t))
    return t


def bump_seed(delta=0x9E3779B97F4A7C1):
    """Advance the step seed on the device (stream-ordered; captured into training graphs)."""
    call("retr_seed_bump", ptr(seed_base()), delta, _st())


_SIDE = {}
# Side-stream overlap switches (A/B-tested by tools/ab_step.py, profiles/r2_ab_side_stream.txt:
# with the whole step in one hipGraph the extra cross-stream edges cost more than the overlap
# gains, so both are off by default): transformer blocks / backbone.
OVERLAP = {"transformer": False, "backbone": False}


class _Overlap:
    """Weight-gradient GEMMs on a second stream, overlapping the data-gradient chain of the
    same backward Function (both are short, latency-bound launches at the transformer's
    shapes).  ``side()`` forks the side stream from everything issued so far on the current
    stream; ``join()`` makes the current stream wait for the side work before the Function
    returns its gradients, so autograd, the caching allocator and graph capture (the side
    branch rejoins the capture stream) see ordinary single-stream semantics."""

    def __init__(self, enabled=True):
        self.main = torch.cuda.current_stream()
        self.enabled = enabled
        dev = self.main.device
        st = _SIDE.get(dev)
        if st is None:
            st = _SIDE[dev] = torch.cuda.Stream(device=dev)
        self.stream = st
        self.used = False

    def side(self):
        if not self.enabled:
            import contextlib
            return contextlib.nullcontext()
        self.stream.wait_stream(self.main)
        self.used = True
        return torch.cuda.stream(self.stream)

    def join(self):
        if self.used:
            self.main.wait_stream(self.stream)


def set_deterministic(on=True):
    """Fixed-order reductions in every kernel (config.deterministic): weight-gradient GEMMs
    without split-K atomics, ordered bias-gradient column sums.  Process-wide."""
    call("retr_set_deterministic", 1 if on else 0)


def is_deterministic():
    from ._lib import load
    return bool(load().retr_get_deterministic())


def dcode(dtype):
    if dtype == torch.bfloat16:
        return BF16
    if dtype == torch.float32:
        return F32
    raise TypeError(f"unsupported compute dtype {dtype}")


def _st():
    return _lib.stream()


class _WeightCache:
    """Compute-dtype copies of fp32 parameters, refreshed when the parameter changes
    (``_version`` bump after an optimizer step).  Optional zero-padding of rows."""

    ATTR = "_retr_compute_copies"

    def get(self, p, dtype, rows=None):
        rows = rows or p.shape[0]
        if dtype == torch.float32 and rows == p.shape[0] and p.is_contiguous():
            return p.detach()
        sh = getattr(p, "_retr_shadow", None)
        if rows != p.shape[0]:   # FusedAdamW's slot reserves the padding rows (models/caption.py)
            pad = getattr(p, "_retr_pad_shadow", None)
            if sh is None or pad is None or pad.shape[0] != rows:
                sh = None
        if sh is not None and dtype == torch.bfloat16:
            # FusedAdamW's bf16 parameter shadow (written by its update kernel): cast into it
            # only when the parameter changed some other way
            ver = (p._version, p.data_ptr())
            if getattr(p, "_retr_shadow_ver", None) != ver:
                src = p.detach().contiguous()
                call("retr_cast", dcode(dtype), ptr(src), ptr(sh), src.numel(), _st())
                p._retr_shadow_ver = ver
            return sh if rows == p.shape[0] else p._retr_pad_shadow
        key = (dtype, rows)
        ent = getattr(p, self.ATTR, None)   # cache lives on the parameter object itself
        ver = (p._version, p.data_ptr())
        if ent is not None and key in ent and ent[key][0] == ver:
            return ent[key][1]
        src = p.detach().contiguous()
        if ent is not None and key in ent:
            out = ent[key][1]   # same shape: re-cast in place (padding rows stay zero, no fill)
        else:
            out = torch.zeros((rows,) + tuple(p.shape[1:]), dtype=dtype, device=p.device) \
                if rows != p.shape[0] else torch.empty(p.shape, dtype=dtype, device=p.device)
        call("retr_cast", dcode(dtype), ptr(src), ptr(out), src.numel(), _st())
        if ent is None:
            ent = {}
            setattr(p, self.ATTR, ent)
        ent[key] = (ver, out)
        return out

    def get_t(self, p, dtype, rows=None):
        """W^T [K][rows] (compute dtype) of a [N][K...] parameter, rows >= N zero-padded: the
        B operand of the data-gradient GEMM dX = dY W.  By default a view of the row-major
        copy (``get``) that the GEMM reads transposed through LDS (no per-step transpose
        kernels); with DGRAD_TRANSPOSED_COPIES a materialised K-contiguous transpose."""
        if not DGRAD_TRANSPOSED_COPIES:
            return _TView(self.get(p, dtype, rows).reshape(rows or p.shape[0], -1))
        n = p.shape[0]
        rows = rows or n
        key = ("T", dtype, rows)
        ent = getattr(p, self.ATTR, None)
        ver = (p._version, p.data_ptr())
        if ent is not None and key in ent and ent[key][0] == ver:
            return ent[key][1]
        src = p.detach().reshape(n, -1).contiguous()
        k = src.shape[1]
        out = torch.empty(k, rows, dtype=dtype, device=p.device)
        call("retr_transpose_cast", dcode(dtype), ptr(src), ptr(out), n, k, rows, _st())
        if ent is None:
            ent = {}
            setattr(p, self.ATTR, ent)
        ent[key] = (ver, out)
        return out


WEIGHTS = _WeightCache()

# dgrad B operand: False (default) = the row-major weight copy read transposed in LDS
# (ds_read_b64_tr_b16), True = a K-contiguous transposed copy per weight version (one
# transpose_cast launch per weight and step); env RETR_DGRAD_TRANSPOSED=1 for A/B runs
DGRAD_TRANSPOSED_COPIES = os.environ.get("RETR_DGRAD_TRANSPOSED", "0") == "1"


class _TView:
    """W^T of a row-major [N][K] weight copy without materialising it: ``shape`` is (K, N) and
    ``[:, a:b]`` selects rows a:b of W (the in-projection's q/k/v blocks)."""

    def __init__(self, w):
        self.w = w

    @property
    def shape(self):
        return (self.w.shape[1], self.w.shape[0])

    def __getitem__(self, idx):
        rows, cols = idx
        assert rows == slice(None)
        return _TView(self.w[cols])


def _pad_vec(v, n):
    """fp32 copy of ``v`` zero-padded to ``n`` (the vocabulary head's bias): the padded buffer
    lives on the parameter and is refreshed in place (one copy, no fill) when ``v`` changes."""
    if v is None:
        return None
    if v.shape[0] == n:
        return v.detach().contiguous()
    pad = getattr(v, "_retr_pad_data", None)   # FusedAdamW slot with the zero padding rows
    if pad is not None and pad.shape[0] == n and pad.data_ptr() == v.data_ptr():
        return pad
    ver = (v._version, v.data_ptr(), n)
    ent = getattr(v, "_retr_padvec", None)
    if ent is not None and ent[0] == ver:
        return ent[1]
    out = ent[1] if ent is not None and ent[1].shape[0] == n else \
        torch.zeros(n, dtype=torch.float32, device=v.device)
    out[: v.shape[0]].copy_(v.detach())
    v._retr_padvec = (ver, out)
    return out


def _drop_p(module_training, p):
    return float(p) if module_training and p > 0 else 0.0


# ---------------------------------------------------------------------------------------------
# low-level launch wrappers (no autograd)
# ---------------------------------------------------------------------------------------------

def _splits(dtype, M, N, K):
    """Split-K slice count for an M x N output over a K-long reduction (retr_linear_splits)."""
    if dtype != torch.bfloat16:
        return 1
    key = (M, N, K)
    s = _SPLITS.get(key)
    if s is None:
        s = _SPLITS[key] = int(_lib.load().retr_linear_splits(dcode(dtype), M, N, K))
    return s


_SPLITS = {}


def k_linear_fwd(x, w, bias, y, relu=0, res=None, drop_p=0.0, seed=0, ln=None):
    """``ln`` = (gamma, beta, eps, ln_y, ln_y2, pos, period, mean, rstd): also LayerNorm the
    (fp32) output -- in the split-K slab epilogue when the linear splits (retr_linear_fwd_splitk_ln),
    else by a LayerNorm launch after it."""
    M, K = x.shape
    N = w.shape[0]
    splits = _splits(x.dtype, M, N, K)
    if ln is not None and splits > 1:
        g, b, eps, ly, ly2, pos, period, mean, rstd = ln
        posd = pos.detach().contiguous() if pos is not None else None
        ref = ly if ly is not None else ly2
        d = _lib.LnOut(ptr(g), ptr(b), float(eps), int(ref.dtype == torch.bfloat16), ptr(ly),
                       ptr(ly2), ref.stride(0), ptr(posd), int(period or 1), ptr(mean),
                       ptr(rstd))
        ws = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
        call("retr_linear_fwd_splitk_ln", dcode(x.dtype), ptr(x), x.stride(0), ptr(w),
             w.stride(0), ptr(bias), ptr(y), y.stride(0), M, N, K, relu, ptr(res),
             res.stride(0) if res is not None else 0, drop_p, seed, ptr(ws), splits,
             ctypes.byref(d), _st())
        return
    if ln is not None:
        k_linear_fwd(x, w, bias, y, relu, res, drop_p, seed)
        g, b, eps, ly, ly2, pos, period, mean, rstd = ln
        posd = pos.detach().contiguous() if pos is not None else None
        ref = ly if ly is not None else ly2
        call("retr_layernorm_fwd", dcode(ref.dtype), ptr(y), y.stride(0), ptr(g), ptr(b),
             float(eps), M, N, ptr(ly), ref.stride(0), ptr(ly2), ptr(posd), int(period or 1),
             ptr(mean), ptr(rstd), _st())
        return
    if splits > 1:
        # few output tiles, long reduction (FFN down-projection): ordered fp32 slabs + epilogue
        ws = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
        call("retr_linear_fwd_splitk", dcode(x.dtype), ptr(x), x.stride(0), ptr(w), w.stride(0),
             ptr(bias), ptr(y), y.stride(0), int(y.dtype == torch.float32), M, N, K, relu,
             ptr(res), res.stride(0) if res is not None else 0, drop_p, seed, ptr(ws), splits,
             _st())
        return
    call("retr_linear_fwd", dcode(x.dtype), ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(bias),
         ptr(y), y.stride(0), int(y.dtype == torch.float32), M, N, K, relu, ptr(res),
         res.stride(0) if res is not None else 0, drop_p, seed, _st())


def k_linear_dgrad(dy, wt, dx, addend=None, gate=None):
    """dx = gate(dy W [+ addend]) with ``wt`` = W^T [K][N] (see _WeightCache.get_t): a
    materialised transpose, or a _TView of the row-major W [N][K]."""
    M = dy.shape[0]
    K, N = wt.shape
    if isinstance(wt, _TView):
        w, w_trans = wt.w, 0
    else:
        w, w_trans = wt, 1
    splits = _splits(dy.dtype, M, K, N)
    if splits > 1:
        # long reduction, few output tiles (FFN up-projection, the MLP head's vocabulary):
        # fp32 slabs added in order by the epilogue kernel
        ws = torch.empty(splits, M, K, dtype=torch.float32, device=dy.device)
        call("retr_linear_dgrad_splitk", dcode(dy.dtype), ptr(dy), dy.stride(0), ptr(w),
             w.stride(0), ptr(dx), dx.stride(0), int(dx.dtype == torch.float32), M, N, K,
             ptr(addend), int(addend is not None and addend.dtype == torch.float32),
             addend.stride(0) if addend is not None else 0, ptr(gate),
             gate.stride(0) if gate is not None else 0, w_trans, ptr(ws), splits, _st())
        return
    call("retr_linear_dgrad", dcode(dy.dtype), ptr(dy), dy.stride(0), ptr(w), w.stride(0),
         ptr(dx), dx.stride(0), int(dx.dtype == torch.float32), M, N, K, ptr(addend),
         int(addend is not None and addend.dtype == torch.float32),
         addend.stride(0) if addend is not None else 0, ptr(gate),
         gate.stride(0) if gate is not None else 0, w_trans, _st())


def k_linear_wgrad(dy, x, dw, db=None, accumulate=False):
    """dw (=|+=) dy^T x and, fused, db (=|+=) colsum(dy); overwrite needs no pre-zeroing."""
    M = dy.shape[0]
    N = dw.shape[0]
    K = x.shape[1]
    call("retr_linear_wgrad", dcode(dy.dtype), ptr(dy), dy.stride(0), ptr(x), x.stride(0),
         ptr(dw), dw.stride(0), M, N, K, ptr(db), int(accumulate), _st())


def k_linear_fwd_group(items):
    """One launch for independent projections: items of (x, w, bias, y[, relu, res, drop_p,
    seed]); every y has the same dtype (csrc/linear_group.hip)."""
    n = len(items)
    arr = (_lib.LinearFwdDesc * n)()
    for i, it in enumerate(items):
        x, w, bias, y = it[:4]
        relu, res, drop_p, seed = (tuple(it[4:]) + (0, None, 0.0, 0)[len(it) - 4:])
        d = arr[i]
        d.x, d.ldx, d.w, d.ldw = ptr(x), x.stride(0), ptr(w), w.stride(0)
        d.bias, d.y, d.ldy = ptr(bias), ptr(y), y.stride(0)
        d.residual, d.ldr = ptr(res), res.stride(0) if res is not None else 0
        d.drop_p, d.seed = drop_p, seed
        d.M, d.N, d.K, d.relu = x.shape[0], w.shape[0], x.shape[1], relu
    y0 = items[0][3]
    call("retr_linear_fwd_group", dcode(items[0][0].dtype), int(y0.dtype == torch.float32), n,
         arr, _st())


def k_linear_dgrad_group(items):
    """One launch for independent data gradients: items of (dy, wt, dx[, addend, gate]) with
    wt as in k_linear_dgrad (all _TView or all materialised)."""
    n = len(items)
    arr = (_lib.LinearDgradDesc * n)()
    w_trans = None
    for i, it in enumerate(items):
        dy, wt, dx = it[:3]
        addend = it[3] if len(it) > 3 else None
        gate = it[4] if len(it) > 4 else None
        K, N = wt.shape
        if isinstance(wt, _TView):
            w, wtr = wt.w, 0
        else:
            w, wtr = wt, 1
        assert w_trans is None or w_trans == wtr, "dgrad group: mixed weight layouts"
        w_trans = wtr
        d = arr[i]
        d.dy, d.lddy, d.w, d.ldw = ptr(dy), dy.stride(0), ptr(w), w.stride(0)
        d.dx, d.lddx = ptr(dx), dx.stride(0)
        d.addend, d.lda = ptr(addend), addend.stride(0) if addend is not None else 0
        d.gate, d.ldg = ptr(gate), gate.stride(0) if gate is not None else 0
        d.M, d.N, d.K = dy.shape[0], N, K
    dx0, a0 = items[0][2], items[0][3] if len(items[0]) > 3 else None
    call("retr_linear_dgrad_group", dcode(items[0][0].dtype), int(dx0.dtype == torch.float32),
         int(a0 is not None and a0.dtype == torch.float32), w_trans, n, arr, _st())


def k_linear_wgrad_group(items, extra=()):
    """One GEMM launch + one ordered slab-sum launch for the weight (and bias) gradients of
    several projections: items of (dy, x, dw, db, accumulate).  ``extra``: further partial-row
    sums (parts, stride, nparts, cols, dst, accumulate) folded into the same slab-sum launch
    (the block's LayerNorm dgamma / dbeta partials, _ln_bwd_fused)."""
    n = len(items)
    arr = (_lib.LinearWgradDesc * n)()
    for i, (dy, x, dw, db, acc) in enumerate(items):
        d = arr[i]
        d.dy, d.lddy, d.x, d.ldx = ptr(dy), dy.stride(0), ptr(x), x.stride(0)
        d.dw, d.lddw, d.db = ptr(dw), dw.stride(0), ptr(db)
        d.M, d.N, d.K, d.accumulate = dy.shape[0], dw.shape[0], x.shape[1], int(acc)
    nbytes = _lib.load().retr_linear_wgrad_group_workspace(n, arr)
    ws = torch.empty(max(1, nbytes // 4), dtype=torch.float32, device=items[0][0].device)
    if not extra:
        call("retr_linear_wgrad_group", dcode(items[0][0].dtype), n, arr, ptr(ws), _st())
        return
    xa = (_lib.SlabSumDesc * len(extra))()
    for i, (parts, stride, nparts, cols, dst, acc) in enumerate(extra):
        xa[i].parts, xa[i].stride, xa[i].nparts = ptr(parts), stride, nparts
        xa[i].cols, xa[i].dst, xa[i].accumulate = cols, ptr(dst), int(acc)
    call("retr_linear_wgrad_group2", dcode(items[0][0].dtype), n, arr, ptr(ws), len(extra), xa,
         _st())


# Deferred weight gradients (bf16 transformer blocks).  A block's backward needs only the DATA
# gradient to go on; its weight / bias gradients (and its LayerNorm dgamma / dbeta partial-row
# sums) are queued and run later as ONE retr_linear_wgrad_batch launch over every queued
# problem: with a whole transformer's projections in one grid (~1000 128x128 tiles) the token
# reduction is not split, so no fp32 slabs and no slab-sum launches (the per-block group path
# splits each block's 80-100 tiles 8-16 ways to fill the chip).  The queue is flushed
#   * at the end of the backward pass (autograd final callback, armed by the first enqueue),
#   * by ddp.GradSync before a gradient bucket is all-reduced (or copied out),
#   * explicitly (flush_wgrad(); engine.forward_backward calls it after backward()).
# Only gradients handed out by FusedAdamW's arena are deferred: autograd adopts those views as
# p.grad without reading them (an accumulating p.grad would read the buffer at once).  Every
# output element is one fp32 chain over all tokens in order, so the bits do not depend on where
# the flushes fall (segmented DP capture == single graph).
WGRAD_DEFER = True
_WQ = []            # [(descs, extras, keepalive, dst ranges)]
_WQ_STATE = {"armed": False, "ranges": []}
WGRAD_STATS = {"flushes": 0, "problems": 0}


def _wq_dst_ranges(wg, extra):
    out = []
    for dy, x, dw, db, _ in wg:
        out.append((dw.data_ptr(), dw.data_ptr() + dw.shape[0] * dw.stride(0) * 4))
        if db is not None:
            out.append((db.data_ptr(), db.data_ptr() + db.numel() * 4))
    for (_, _, _, cols, dst, _) in extra:
        out.append((dst.data_ptr(), dst.data_ptr() + cols * 4))
    return out


def _wgrad(wg, extra, arena_ok):
    """Weight gradients of one block: queued (see WGRAD_DEFER) or one grouped launch now."""
    if not (WGRAD_DEFER and arena_ok and wg and wg[0][0].dtype == torch.bfloat16):
        k_linear_wgrad_group(wg, extra) if extra else k_linear_wgrad_group(wg)
        return
    rng = _wq_dst_ranges(wg, extra)
    # two queued problems accumulating into one buffer would race inside the batch launch
    if any(a < d and c < b for a, b in rng for c, d in _WQ_STATE["ranges"]):
        flush_wgrad()
    descs = []
    keep = []
    for dy, x, dw, db, acc in wg:
        descs.append((ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(dw), dw.stride(0), ptr(db),
                      dy.shape[0], dw.shape[0], x.shape[1], int(acc)))
        keep += [dy, x]
    xs = []
    for (parts, stride, nparts, cols, dst, acc) in extra:
        xs.append((ptr(parts), stride, nparts, cols, ptr(dst), int(acc)))
        keep.append(parts)
    _WQ.append((descs, xs, keep))
    _WQ_STATE["ranges"] += rng
    if not _WQ_STATE["armed"]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(flush_wgrad)
            _WQ_STATE["armed"] = True
        except RuntimeError:        # not inside a backward pass: nothing would flush later
            flush_wgrad()


# the MLP head's weight gradients join the deferred batch too (else: one launch each + a
# column-sum launch for the vocabulary bias)
HEAD_WGRAD_DEFER = True

# The fence's flush on a side stream, overlapping the backbone backward: measured 0.3 ms/step
# SLOWER in the graphed cfg2 step (profiles/r4_ab_wgrad_defer.txt), so off by default
WGRAD_SIDE = False
_SIDE = {"stream": None, "pending": False}


def _side_stream(dev):
    st = _SIDE["stream"]
    if st is None or st.device != dev:
        st = _SIDE["stream"] = torch.cuda.Stream(device=dev)
    return st


def join_side():
    """Make the current stream wait for a weight-gradient batch running on the side stream."""
    if _SIDE["pending"]:
        torch.cuda.current_stream(_SIDE["stream"].device).wait_stream(_SIDE["stream"])
        _SIDE["pending"] = False


def flush_wgrad(side=False):
    """Run every queued weight gradient (one launch) and, unless ``side``, wait for any batch
    still running on the side stream.  ``side``: launch on the side stream (forked from the
    current one), so the batch overlaps the kernels that follow until the next join."""
    if not side:
        _WQ_STATE["armed"] = False
    flush_pos()
    if _WQ:
        descs = [d for q in _WQ for d in q[0]]
        xs = [x for q in _WQ for x in q[1]]
        keep = [t for q in _WQ for t in q[2]]
        _WQ.clear()
        _WQ_STATE["ranges"] = []
        dev = keep[0].device
        if side:
            st = _side_stream(dev)
            st.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(st):
                for t in keep:
                    t.record_stream(st)
                _wgrad_batch_launch(descs, xs, dev)
            _SIDE["pending"] = True
        else:
            _wgrad_batch_launch(descs, xs, dev)
        WGRAD_STATS["flushes"] += 1
        WGRAD_STATS["problems"] += len(descs)
        del keep
    if not side:
        join_side()


class _WgradFence(torch.autograd.Function):
    """Identity on the transformer's input rows: its backward runs once every transformer block
    has queued its weight gradients, and starts their batch (on the side stream with
    WGRAD_SIDE) while the backbone backward proceeds."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        flush_wgrad(side=WGRAD_SIDE)
        return g


def wgrad_fence(x):
    return _WgradFence.apply(x) if x.requires_grad and torch.is_grad_enabled() else x


def _wgrad_batch_launch(descs, xs, dev):
    n, nx = len(descs), len(xs)
    arr = (_lib.LinearWgradDesc * max(1, n))()
    for i, (dy, lddy, x, ldx, dw, lddw, db, M, N, K, acc) in enumerate(descs):
        d = arr[i]
        d.dy, d.lddy, d.x, d.ldx, d.dw, d.lddw, d.db = dy, lddy, x, ldx, dw, lddw, db
        d.M, d.N, d.K, d.accumulate = M, N, K, acc
    xa = (_lib.SlabSumDesc * max(1, nx))()
    for i, (parts, stride, nparts, cols, dst, acc) in enumerate(xs):
        xa[i].parts, xa[i].stride, xa[i].nparts = parts, stride, nparts
        xa[i].cols, xa[i].dst, xa[i].accumulate = cols, dst, acc
    nbytes = int(_lib.load().retr_linear_wgrad_batch_table_bytes(n, nx))
    table = torch.empty((nbytes + 15) // 16 * 16, dtype=torch.uint8, device=dev)
    call("retr_linear_wgrad_batch", n, arr, nx, xa, ptr(table), table.numel(), _st())


def k_linear_wgrad_batch(items, extra=()):
    """One retr_linear_wgrad_batch launch now: items of (dy, x, dw, db, accumulate) as in
    k_linear_wgrad_group, any number of them; ``extra`` partial-row sums likewise."""
    descs = [(ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(dw), dw.stride(0), ptr(db),
              dy.shape[0], dw.shape[0], x.shape[1], int(acc)) for dy, x, dw, db, acc in items]
    xs = [(ptr(parts), stride, nparts, cols, ptr(dst), int(acc))
          for (parts, stride, nparts, cols, dst, acc) in extra]
    _wgrad_batch_launch(descs, xs, items[0][0].device)


def wgrad_pending():
    return len(_WQ)


def _empty(*shape, dev):
    return torch.empty(shape, dtype=torch.float32, device=dev)


def k_bias_grad(dy, db, N=None):
    call("retr_bias_grad", dcode(dy.dtype), ptr(dy), dy.stride(0), dy.shape[0], N or db.shape[0],
         ptr(db), _st())


def k_dropout_apply(x, y, drop_p, seed):
    """y = x * keep * 1/(1-p)  (x fp32 [M,N]); plain cast when drop_p == 0."""
    M, N = x.shape
    call("retr_dropout_apply", dcode(y.dtype), ptr(x), x.stride(0), ptr(y), y.stride(0), M, N,
         drop_p, seed, _st())


ATTN_DMASK = True   # save the attention-dropout keep bits in the forward for the backward


def attn_dmask(B, H, Lq, Lk, drop_p, dtype, hd, dev):
    """Buffer for the forward's attention-dropout keep bits (retr_attention_fwd_dm), or None
    when dropout is off or the kernels that use it do not run (bf16, head dim 32 / 64)."""
    if not (ATTN_DMASK and drop_p > 0 and dtype == torch.bfloat16 and hd in (32, 64)):
        return None
    n = _lib.load().retr_attention_dropout_mask_bytes(B, H, Lq, Lk) // 4
    return torch.empty(max(1, n), dtype=torch.int32, device=dev)


def k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, causal, drop_p, seed, lse, probs=None,
                    dmask=None):
    call("retr_attention_fwd_dm", dcode(q.dtype), ptr(q), q.stride(0), ptr(k), k.stride(0),
         ptr(v), v.stride(0), ptr(o), o.stride(0), B, H, Lq, Lk, hd, ptr(kpm), int(causal), drop_p,
         seed, ptr(lse), ptr(probs), ptr(dmask), _st())


def k_attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, hd, kpm, causal, drop_p,
                    seed, dmask=None):
    ws = torch.empty(B * H * Lq, dtype=torch.float32, device=q.device)
    call("retr_attention_bwd_dm", dcode(q.dtype), ptr(q), q.stride(0), ptr(k), k.stride(0),
         ptr(v), v.stride(0), ptr(o), o.stride(0), ptr(do), do.stride(0), ptr(lse), ptr(dq),
         dq.stride(0), ptr(dk), dk.stride(0), ptr(dv), dv.stride(0), B, H, Lq, Lk, hd, ptr(kpm),
         int(causal), drop_p, seed, ptr(ws), ptr(dmask), _st())


def ln_workspace(M, C, dev):
    """fp32 scratch for the LayerNorm backward's per-block dgamma/dbeta partials."""
    n = _lib.load().retr_layernorm_bwd_workspace(M, C) // 4
    return torch.empty(n, dtype=torch.float32, device=dev)


def _rows(t):
    return t.reshape(-1, t.shape[-1]) if t.dim() != 2 else t


# ---------------------------------------------------------------------------------------------
# LayerNorm (+ position add)
# ---------------------------------------------------------------------------------------------

class _LnPos(torch.autograd.Function):
    """mode: 'plain' -> LN(x); 'pos' -> LN(x)+pos; 'both' -> (LN(x), LN(x)+pos)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, pos, period, eps, cdtype, mode):
        _lib.require_device(x)
        M, C = x.shape
        dev = x.device
        got = _ln_take(x, _ln_key(gamma, beta, eps, pos, period, mode in ("plain", "both"),
                                  mode in ("pos", "both"), cdtype))
        if got is not None:
            y, y2, mean, rstd = got
        else:
            y = torch.empty(M, C, dtype=cdtype, device=dev) if mode in ("plain", "both") else None
            y2 = torch.empty(M, C, dtype=cdtype, device=dev) if mode in ("pos", "both") else None
            mean = torch.empty(M, dtype=torch.float32, device=dev)
            rstd = torch.empty_like(mean)
            posd = pos.detach().contiguous() if pos is not None else None
            call("retr_layernorm_fwd", dcode(cdtype), ptr(x), x.stride(0), ptr(gamma),
                 ptr(beta), float(eps), M, C, ptr(y), C, ptr(y2), ptr(posd), int(period or 1),
                 ptr(mean), ptr(rstd), _st())
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.gparams = (gamma, beta, pos)
        ctx.period = period
        ctx.mode = mode
        ctx.pos_shape = tuple(pos.shape) if pos is not None else None
        if mode == "both":
            return y, y2
        return y if mode == "plain" else y2

    @staticmethod
    def backward(ctx, *grads):
        x, gamma, mean, rstd = ctx.saved_tensors
        mode = ctx.mode
        if mode == "both":
            dy, dy2 = grads
        elif mode == "plain":
            dy, dy2 = grads[0], None
        else:
            dy, dy2 = None, grads[0]
        M, C = x.shape
        dx = torch.empty(M, C, dtype=torch.float32, device=x.device)
        gp, bp, pp = ctx.gparams
        dgamma, _ = grad_buffer(gp)
        dbeta, _ = grad_buffer(bp)
        if dy is not None:
            dy = dy.contiguous()
        if dy2 is not None:
            dy2 = dy2.contiguous()
            if dy is not None and dy.dtype != dy2.dtype:
                dy2 = dy2.to(dy.dtype)
        ref = dy if dy is not None else dy2
        ws = ln_workspace(M, C, x.device)
        call("retr_layernorm_bwd", dcode(ref.dtype), ptr(dy), ptr(dy2), C, ptr(x), x.stride(0),
             ptr(gamma), ptr(mean), ptr(rstd), M, C, ptr(dx), dx.stride(0), None, ptr(dgamma),
             ptr(dbeta), ptr(ws), _st())
        dpos = None
        if ctx.pos_shape is not None and ctx.needs_input_grad[3] and dy2 is not None:
            dpos, _ = grad_buffer(pp)
            call("retr_pos_grad", dcode(dy2.dtype), ptr(dy2), dy2.stride(0), M, C, ctx.period,
                 ptr(dpos), _st())
        return dx, dgamma, dbeta, dpos, None, None, None, None


def ln_pos(x, norm, cdtype, pos=None, period=None, mode=None, eps=None):
    """LayerNorm(x) in compute dtype; with ``pos`` also LayerNorm(x) + pos[row % period]."""
    if mode is None:
        mode = "plain" if pos is None else "both"
    return _LnPos.apply(x, norm.weight, norm.bias, pos, period,
                        norm.eps if eps is None else eps, cdtype, mode)


# LayerNorm of a residual-stream tensor produced by the epilogue of the linear that wrote it
# (retr_linear_fwd_splitk_ln: the FFN down-projection's slab epilogue also normalises its output
# for the next pre-norm block or the stack's final norm).  The producer tags its output with
# (key, version, (LN(x), LN(x)+pos, mean, rstd)); the consumer's _ln_fwd takes the tag when the
# key (the same norm parameters, eps, position table, period and outputs) and the version match,
# else it launches the LayerNorm as before.  Same bits either way.
FUSE_LN_NEXT = True
LN_NEXT_STATS = {"hit": 0, "miss": 0}


def _ln_key(gamma, beta, eps, pos, period, plain, with_pos, cdtype):
    return (id(gamma), id(beta), float(eps), id(pos) if pos is not None else None,
            int(period or 1) if pos is not None else 1, bool(plain), bool(with_pos), cdtype)


def _ln_take(x, key):
    ent = getattr(x, "_retr_ln", None)
    if ent is None:
        return None
    x._retr_ln = None
    if ent[0] == key and ent[1] == x._version:
        LN_NEXT_STATS["hit"] += 1
        return ent[2]
    LN_NEXT_STATS["miss"] += 1
    return None


def _ln_fwd(x, gamma, beta, eps, cdtype, pos=None, period=1, plain=True, with_pos=False):
    """LayerNorm kernel: (LN(x) | None, LN(x)+pos[row % period] | None, mean, rstd)."""
    got = _ln_take(x, _ln_key(gamma, beta, eps, pos, period, plain, with_pos, cdtype))
    if got is not None:
        return got
    M, C = x.shape
    dev = x.device
    y = torch.empty(M, C, dtype=cdtype, device=dev) if plain else None
    y2 = torch.empty(M, C, dtype=cdtype, device=dev) if with_pos else None
    mean = torch.empty(M, dtype=torch.float32, device=dev)
    rstd = torch.empty_like(mean)
    posd = pos.detach().contiguous() if pos is not None else None
    call("retr_layernorm_fwd", dcode(cdtype), ptr(x), x.stride(0), ptr(gamma), ptr(beta),
         float(eps), M, C, ptr(y), C, ptr(y2), ptr(posd), int(period or 1), ptr(mean),
         ptr(rstd), _st())
    return y, y2, mean, rstd


def _ln_bwd(x, gamma, beta, mean, rstd, dy, dy2, addend, pos=None, period=1, need_dpos=False):
    """dx = addend + LN'(dy + dy2) (fp32), dgamma/dbeta into their gradient buffers, and the
    position gradient (rows summed by row % period) when ``need_dpos``."""
    M, C = x.shape
    ref = dy if dy is not None else dy2
    if dy is not None and dy2 is not None and dy.dtype != dy2.dtype:
        dy2 = dy2.to(dy.dtype)
    dx = torch.empty(M, C, dtype=torch.float32, device=x.device)
    dgamma, _ = grad_buffer(gamma)
    dbeta, _ = grad_buffer(beta)
    ws = ln_workspace(M, C, x.device)
    call("retr_layernorm_bwd", dcode(ref.dtype), ptr(dy), ptr(dy2), C, ptr(x), x.stride(0),
         ptr(gamma), ptr(mean), ptr(rstd), M, C, ptr(dx), dx.stride(0), ptr(addend),
         ptr(dgamma), ptr(dbeta), ptr(ws), _st())
    dpos = None
    if need_dpos and dy2 is not None:
        dpos, _ = grad_buffer(pos)
        call("retr_pos_grad", dcode(dy2.dtype), ptr(dy2), dy2.stride(0), M, C, int(period),
             ptr(dpos), _st())
    return dx, dgamma, dbeta, dpos


# Fused backward of the transformer blocks (bf16 compute): a block's LayerNorm backward also
#  * writes the bf16 dropout(dx) of the residual dropout of the block that produced its input --
#    exactly that block's first backward launch (retr_dropout_apply of its incoming gradient),
#    which then finds it in _DBR instead of launching it;
#  * leaves its dgamma / dbeta partial rows for the block's weight-gradient slab sum instead of
#    a separate reduction launch.
_DBR = {}   # data_ptr of dx -> ((drop_p, seed) of the producing block, dx._version, bf16 copy)
FUSE_LN_BWD = True   # tests switch the fused path off to compare against the unfused launches
FUSE_LN_PARAMS = True   # dgamma / dbeta partials into the wgrad slab sum (else their own launch)
DBR_STATS = {"hit": 0, "miss": 0}


# Gradients of a tensor several blocks read (the decoder's query positions: 12 blocks; the
# encoder memory and its positional sum: the 6 cross-attention blocks): every contributor adds
# into ONE buffer in its own kernel (retr_pos_grad adds; the data-gradient GEMM epilogue takes
# the buffer as addend) and only the last one in backward order returns it -- instead of a
# zero-filled buffer per block and autograd's pairwise adds.
_SHARED = {}   # id(tensor) -> [contributors left, buffer or None]


def begin_pass():
    """Forget the previous pass's unused fused dropout-gradient copies and shared gradients
    (and run any weight gradient still queued: a backward that never reached its end)."""
    _DBR.clear()
    _SHARED.clear()
    flush_wgrad()


def _share(t):
    """Forward: one more block will contribute to the gradient of ``t``."""
    e = _SHARED.get(id(t))
    if e is None:
        _SHARED[id(t)] = e = [0, None, t]
    e[0] += 1


def _shared_grad(t, make):
    """Backward: (buffer, first, last) -- the shared gradient buffer of ``t`` (made by ``make``
    for its first contributor) and whether this contributor is the first / last one; an
    unregistered ``t`` gets a buffer of its own (first = last = True)."""
    e = _SHARED.get(id(t))
    if e is None or e[0] <= 0:
        return make(), True, True
    first = e[1] is None
    if first:
        e[1] = make()
    e[0] -= 1
    last = e[0] == 0
    buf = e[1]
    if last:
        del _SHARED[id(t)]
    return buf, first, last


def _tag_drop(out, drop_p, seed):
    """Mark a block's fp32 output with its residual dropout (read by the next block)."""
    out._retr_drop = (float(drop_p), int(seed))
    return out


def _take_dbr(dout, drop_p, seed, cdtype):
    """bf16 dropout(dout) for a block's residual dropout: the copy the following block's fused
    LayerNorm backward wrote (same pointer, unmodified since: version check), else one
    retr_dropout_apply launch."""
    ent = _DBR.pop(dout.data_ptr(), None)
    if (ent is not None and ent[0] == (float(drop_p), int(seed)) and ent[1] == dout._version
            and ent[2].shape == dout.shape and ent[2].dtype == cdtype):
        DBR_STATS["hit"] += 1
        return ent[2]
    DBR_STATS["miss"] += 1
    dbr = torch.empty(dout.shape, dtype=cdtype, device=dout.device)
    k_dropout_apply(dout, dbr, drop_p, seed)
    return dbr


def _ln_bwd_fused(x, gamma, beta, mean, rstd, dy, dy2, addend, prev, cdtype, pos=None, period=1,
                  need_dpos=False, slabs=None):
    """_ln_bwd for the bf16 blocks: returns (dx, dgamma, dbeta, dpos, extra, arena) where
    ``extra`` are the dgamma / dbeta partial-row sums for the block's weight-gradient launch and
    ``arena`` says both parameter gradients are FusedAdamW arena views; with ``prev`` = (drop_p,
    seed) of the block that produced x, also caches bf16 dropout(dx) for that block."""
    import ctypes
    M, C = x.shape
    ref = dy if dy is not None else (dy2 if dy2 is not None else x)
    if dy is not None and dy2 is not None and dy.dtype != dy2.dtype:
        dy2 = dy2.to(dy.dtype)
    dx = torch.empty(M, C, dtype=torch.float32, device=x.device)
    dgamma, ag = grad_buffer(gamma)
    dbeta, ab = grad_buffer(beta)
    ws = ln_workspace(M, C, x.device)
    dxd = torch.empty(M, C, dtype=cdtype, device=x.device) if prev is not None else None
    nparts = ctypes.c_int(0)
    if slabs is not None:
        # dy = bf16(sum of the producing data gradient's split-K slabs), summed here
        sws, nsl = slabs
        call("retr_layernorm_bwd_slabs", ptr(sws), nsl, ptr(x), x.stride(0), ptr(gamma),
             ptr(mean), ptr(rstd), M, C, ptr(dx), dx.stride(0), ptr(addend), ptr(dgamma),
             ptr(dbeta), ptr(ws), ptr(dxd), C, prev[0] if prev else 0.0, prev[1] if prev else 0,
             ctypes.addressof(nparts) if FUSE_LN_PARAMS else None, _st())
    else:
        call("retr_layernorm_bwd2", dcode(ref.dtype), ptr(dy), ptr(dy2), C, ptr(x),
             x.stride(0), ptr(gamma), ptr(mean), ptr(rstd), M, C, ptr(dx), dx.stride(0),
             ptr(addend), ptr(dgamma), ptr(dbeta), ptr(ws), ptr(dxd), C,
             prev[0] if prev else 0.0, prev[1] if prev else 0,
             ctypes.addressof(nparts) if FUSE_LN_PARAMS else None, _st())
    if dxd is not None:
        _DBR[dx.data_ptr()] = (prev, dx._version, dxd)
    n = nparts.value
    extra = [(ws, 2 * C, n, C, dgamma, 1), (ws[C:], 2 * C, n, C, dbeta, 1)] if n > 0 else []
    dpos = None
    if need_dpos and dy2 is not None:
        dpos, _, last = _shared_grad(pos, lambda: grad_buffer(pos))
        dpos, arena = dpos
        if POS_DEFER and arena and dy2.dtype == torch.bfloat16:
            _pos_queue(dy2, M, C, int(period), dpos)
        else:
            call("retr_pos_grad", dcode(dy2.dtype), ptr(dy2), dy2.stride(0), M, C, int(period),
                 ptr(dpos), _st())        # adds into the (zeroed or shared) buffer
        if not last:
            dpos = None
    return dx, dgamma, dbeta, dpos, extra, ag and ab


# Position gradients of a table several blocks read (the decoder's query positions: 12 blocks,
# plus the DecoderEmbeddings sum, which joins the same shared buffer: _EmbedLN) are queued per
# buffer and summed by one retr_pos_grad_multi launch when the weight-gradient queue flushes, or
# when the table's last contributor (the embedding backward) needs the buffer (same sums in the
# same order as one retr_pos_grad per block).  Only for FusedAdamW arena buffers, which autograd
# adopts as .grad without reading them -- and only because the queue holds the buffer's ADDRESS,
# never the tensor: an extra reference makes AccumulateGrad clone the buffer (a read, in stream
# order before the queued sums land; round 4's lost query-position gradient).
POS_DEFER = True    # graphed step 9.670 -> 9.622 ms (profiles/r4_ab_pos_defer.txt)
_POSQ = {}     # dpos data_ptr -> [dpos data_ptr, C, period, [(dy2, M), ...]]


def _pos_queue(dy2, M, C, period, dpos):
    p = dpos.data_ptr()
    e = _POSQ.get(p)
    if e is None or e[1] != C or e[2] != period:
        if e is not None:
            _pos_flush_one(e)
        e = _POSQ[p] = [p, C, period, []]
    e[3].append((dy2, M))
    if len(e[3]) == 16:
        _pos_flush_one(e)
        del _POSQ[p]
    if not _WQ_STATE["armed"]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(flush_wgrad)
            _WQ_STATE["armed"] = True
        except RuntimeError:
            flush_pos()


def _pos_flush_one(e):
    dpos, C, period, items = e
    arr = (_lib.PosItem * len(items))()
    for i, (d, M) in enumerate(items):
        arr[i].d, arr[i].ld, arr[i].M = ptr(d), d.stride(0), M
    call("retr_pos_grad_multi", BF16, len(items), arr, C, period, dpos, 1, _st())


def flush_pos(addr=None):
    """Run the queued position-gradient sums (only the buffer at ``addr`` if given)."""
    if addr is not None:
        e = _POSQ.pop(addr, None)
        if e is not None:
            _pos_flush_one(e)
        return
    for e in list(_POSQ.values()):
        _pos_flush_one(e)
    _POSQ.clear()


def _deferred_overlaps(lo, hi):
    """True if a queued weight / position gradient writes into the byte range [lo, hi)."""
    if any(a < hi and lo < b for a, b in _WQ_STATE["ranges"]):
        return True
    return any(lo <= p < hi for p in _POSQ)


def _on_grad_reuse(p):
    """optim.grad_buffer hook: parameter ``p``'s arena slot was already handed out this pass
    and a second contributor is asking for a buffer.  Autograd will add the two (InputBuffer /
    AccumulateGrad read the arena view), so whatever is still queued for that slot must be in
    stream order before this contributor's kernels: flush it now."""
    v = p._retr_grad_view
    lo = v.data_ptr()
    hi = lo + v.numel() * v.element_size()
    if _deferred_overlaps(lo, hi):
        GRAD_REUSE_STATS["flushes"] += 1
        flush_wgrad()


GRAD_REUSE_STATS = {"flushes": 0}
_optim.REUSE_HOOK = _on_grad_reuse


# ---------------------------------------------------------------------------------------------
# attention sub-layers
# ---------------------------------------------------------------------------------------------

class _SelfAttnBlock(torch.autograd.Function):
    """x_new = x + drop(out_proj(MHA(q=k=LN(x)+pos, v=LN(x))))  — SelfAttResidual
    (models/transformer_modules.py:22-46) with its pre-norm inside the Function: the
    backward returns dx = dout + LN'(dnpos + dn) in one LayerNorm-backward pass (no separate
    residual-gradient add)."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, pos, period, eps, w_in, b_in, w_out, b_out, B, L, H, kpm,
                causal, drop_attn, drop_res, cdtype, want_probs):
        _lib.require_device(x)
        n, npos, mean, rstd = _ln_fwd(x, ln_w, ln_b, eps, cdtype, pos, period, True, True)
        res = x
        M, C = n.shape
        hd = C // H
        win = WEIGHTS.get(w_in, cdtype)
        wout = WEIGHTS.get(w_out, cdtype)
        dev = n.device
        qk = torch.empty(M, 2 * C, dtype=cdtype, device=dev)
        v = torch.empty(M, C, dtype=cdtype, device=dev)
        k_linear_fwd_group([(npos, win[: 2 * C], b_in[: 2 * C].detach(), qk),
                            (n, win[2 * C:], b_in[2 * C:].detach(), v)])
        o = torch.empty(M, C, dtype=cdtype, device=dev)
        lse = torch.empty(B * H * L, dtype=torch.float32, device=dev)
        s_att, s_res = next_seed(), next_seed()
        probs = torch.empty(B, L, L, dtype=torch.float32, device=dev) if want_probs else None
        dmask = attn_dmask(B, H, L, L, drop_attn, cdtype, hd, dev)
        k_attention_fwd(qk[:, :C], qk[:, C:], v, o, B, H, L, L, hd, kpm, causal, drop_attn,
                        s_att, lse, probs, dmask)
        ctx.dmask = dmask
        out = torch.empty(M, C, dtype=torch.float32, device=dev)
        k_linear_fwd(o, wout, b_out.detach(), out, res=res, drop_p=drop_res, seed=s_res)
        ctx.save_for_backward(npos, n, qk, v, o, lse, kpm, w_in, w_out, x, ln_w, mean, rstd)
        ctx.gparams = (w_in, b_in, w_out, b_out)
        ctx.ln = (ln_w, ln_b, pos, period)
        ctx.cfg = (B, L, H, causal, drop_attn, drop_res, s_att, s_res, cdtype)
        ctx.prev = getattr(x, "_retr_drop", None)
        _tag_drop(out, drop_res, s_res)
        if cdtype == torch.bfloat16 and FUSE_LN_BWD and pos is not None and pos.requires_grad:
            _share(pos)
        if want_probs:
            ctx.mark_non_differentiable(probs)
            return out, probs
        return out

    @staticmethod
    def backward(ctx, dout, dprobs=None):
        npos, n, qk, v, o, lse, kpm, w_in, w_out, x, ln_w, mean, rstd = ctx.saved_tensors
        B, L, H, causal, drop_attn, drop_res, s_att, s_res, cdtype = ctx.cfg
        M, C = n.shape
        hd = C // H
        dev = n.device
        dout = dout.contiguous()
        wint = WEIGHTS.get_t(w_in, cdtype)
        woutt = WEIGHTS.get_t(w_out, cdtype)
        fused = cdtype == torch.bfloat16 and FUSE_LN_BWD
        if fused:
            dbr = _take_dbr(dout, drop_res, s_res, cdtype)
        else:
            dbr = torch.empty(M, C, dtype=cdtype, device=dev)
            k_dropout_apply(dout, dbr, drop_res, s_res)
        (dw_in, a0), (db_in, a1), (dw_out, a2), (db_out, a3) = map(grad_buffer, ctx.gparams)
        arena = a0 and a1 and a2 and a3
        do = torch.empty(M, C, dtype=cdtype, device=dev)
        k_linear_dgrad(dbr, woutt, do)
        dqk = torch.empty(M, 2 * C, dtype=cdtype, device=dev)
        dv = torch.empty(M, C, dtype=cdtype, device=dev)
        k_attention_bwd(qk[:, :C], qk[:, C:], v, o, do, lse, dqk[:, :C], dqk[:, C:], dv, B, H,
                        L, L, hd, kpm, causal, drop_attn, s_att, ctx.dmask)
        ctx.dmask = None
        dnpos = torch.empty(M, C, dtype=cdtype, device=dev)
        dn = torch.empty(M, C, dtype=cdtype, device=dev)
        k_linear_dgrad_group([(dqk, wint[:, : 2 * C], dnpos), (dv, wint[:, 2 * C:], dn)])
        _, ln_b, pos, period = ctx.ln
        # the block's three weight gradients (+ biases): one grouped GEMM + one slab sum (with
        # the LayerNorm's parameter partials in it on the fused path)
        wg = [(dbr, o, dw_out, db_out, True), (dqk, npos, dw_in[: 2 * C], db_in[: 2 * C], True),
              (dv, n, dw_in[2 * C:], db_in[2 * C:], True)]
        if fused:
            dx, dlw, dlb, dpos, extra, la = _ln_bwd_fused(x, ln_w, ln_b, mean, rstd, dn, dnpos,
                                                          dout, ctx.prev, cdtype, pos, period,
                                                          ctx.needs_input_grad[3])
            _wgrad(wg, extra, arena and la)
        else:
            k_linear_wgrad_group(wg)
            dx, dlw, dlb, dpos = _ln_bwd(x, ln_w, ln_b, mean, rstd, dn, dnpos, dout, pos, period,
                                         ctx.needs_input_grad[3])
        return (dx, dlw, dlb, dpos, None, None, dw_in, db_in, dw_out, db_out) + (None,) * 9


class _CrossAttnBlock(torch.autograd.Function):
    """y_new = y + drop(out_proj(MHA(q=LN(y)+qpos, k=mem_pos, v=mem)))  — CrossAttResidual
    (models/transformer_modules.py:49-74) with its pre-norm inside the Function (see
    _SelfAttnBlock)."""

    @staticmethod
    def forward(ctx, y, ln_w, ln_b, qp, period, eps, mem_pos, mem, w_in, b_in, w_out, b_out, B,
                Lq, Lk, H, kpm, drop_attn, drop_res, cdtype, want_probs):
        _lib.require_device(y)
        _, qpos, mean, rstd = _ln_fwd(y, ln_w, ln_b, eps, cdtype, qp, period, False, True)
        res = y
        Mq, C = qpos.shape
        Mk = mem.shape[0]
        hd = C // H
        win = WEIGHTS.get(w_in, cdtype)
        wout = WEIGHTS.get(w_out, cdtype)
        dev = qpos.device
        q = torch.empty(Mq, C, dtype=cdtype, device=dev)
        k = torch.empty(Mk, C, dtype=cdtype, device=dev)
        v = torch.empty(Mk, C, dtype=cdtype, device=dev)
        k_linear_fwd_group([(qpos, win[:C], b_in[:C].detach(), q),
                            (mem_pos, win[C: 2 * C], b_in[C: 2 * C].detach(), k),
                            (mem, win[2 * C:], b_in[2 * C:].detach(), v)])
        o = torch.empty(Mq, C, dtype=cdtype, device=dev)
        lse = torch.empty(B * H * Lq, dtype=torch.float32, device=dev)
        s_att, s_res = next_seed(), next_seed()
        probs = torch.empty(B, Lq, Lk, dtype=torch.float32, device=dev) if want_probs else None
        dmask = attn_dmask(B, H, Lq, Lk, drop_attn, cdtype, hd, dev)
        k_attention_fwd(q, k, v, o, B, H, Lq, Lk, hd, kpm, False, drop_attn, s_att, lse, probs,
                        dmask)
        ctx.dmask = dmask
        out = torch.empty(Mq, C, dtype=torch.float32, device=dev)
        k_linear_fwd(o, wout, b_out.detach(), out, res=res, drop_p=drop_res, seed=s_res)
        ctx.save_for_backward(qpos, mem_pos, mem, q, k, v, o, lse, kpm, w_in, w_out, y, ln_w,
                              mean, rstd)
        ctx.gparams = (w_in, b_in, w_out, b_out)
        ctx.ln = (ln_w, ln_b, qp, period)
        ctx.cfg = (B, Lq, Lk, H, drop_attn, drop_res, s_att, s_res, cdtype)
        ctx.prev = getattr(y, "_retr_drop", None)
        _tag_drop(out, drop_res, s_res)
        ctx.shared = cdtype == torch.bfloat16 and FUSE_LN_BWD
        if ctx.shared:
            if qp is not None and qp.requires_grad:
                _share(qp)
            for t in (mem_pos, mem):
                if t.requires_grad:
                    _share(t)
        if want_probs:
            ctx.mark_non_differentiable(probs)
            return out, probs
        return out

    @staticmethod
    def backward(ctx, dout, dprobs=None):
        qpos, mem_pos, mem, q, k, v, o, lse, kpm, w_in, w_out, y, ln_w, mean, rstd = \
            ctx.saved_tensors
        B, Lq, Lk, H, drop_attn, drop_res, s_att, s_res, cdtype = ctx.cfg
        Mq, C = qpos.shape
        Mk = mem.shape[0]
        hd = C // H
        dev = qpos.device
        dout = dout.contiguous()
        wint = WEIGHTS.get_t(w_in, cdtype)
        woutt = WEIGHTS.get_t(w_out, cdtype)
        fused = cdtype == torch.bfloat16 and FUSE_LN_BWD
        if fused:
            dbr = _take_dbr(dout, drop_res, s_res, cdtype)
        else:
            dbr = torch.empty(Mq, C, dtype=cdtype, device=dev)
            k_dropout_apply(dout, dbr, drop_res, s_res)
        (dw_in, a0), (db_in, a1), (dw_out, a2), (db_out, a3) = map(grad_buffer, ctx.gparams)
        arena = a0 and a1 and a2 and a3
        do = torch.empty(Mq, C, dtype=cdtype, device=dev)
        k_linear_dgrad(dbr, woutt, do)
        dq = torch.empty(Mq, C, dtype=cdtype, device=dev)
        dk = torch.empty(Mk, C, dtype=cdtype, device=dev)
        dv = torch.empty(Mk, C, dtype=cdtype, device=dev)
        k_attention_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, hd, kpm, False, drop_attn,
                        s_att, ctx.dmask)
        ctx.dmask = None
        dqpos = torch.empty(Mq, C, dtype=cdtype, device=dev)
        if ctx.shared:
            def mk():
                return torch.empty(Mk, C, dtype=cdtype, device=dev)
            dmem_pos, f_mp, l_mp = _shared_grad(mem_pos, mk)
            dmem, f_m, l_m = _shared_grad(mem, mk)
            # later contributors add the earlier ones' sum in the GEMM epilogue (in place)
            k_linear_dgrad_group([(dq, wint[:, :C], dqpos),
                                  (dk, wint[:, C: 2 * C], dmem_pos, None if f_mp else dmem_pos),
                                  (dv, wint[:, 2 * C:], dmem, None if f_m else dmem)])
        else:
            dmem_pos = torch.empty(Mk, C, dtype=cdtype, device=dev)
            dmem = torch.empty(Mk, C, dtype=cdtype, device=dev)
            l_mp = l_m = True
            k_linear_dgrad_group([(dq, wint[:, :C], dqpos), (dk, wint[:, C: 2 * C], dmem_pos),
                                  (dv, wint[:, 2 * C:], dmem)])
        wg = [(dbr, o, dw_out, db_out, True), (dq, qpos, dw_in[:C], db_in[:C], True),
              (dk, mem_pos, dw_in[C: 2 * C], db_in[C: 2 * C], True),
              (dv, mem, dw_in[2 * C:], db_in[2 * C:], True)]
        _, ln_b, qp, period = ctx.ln
        if fused:
            dy, dlw, dlb, dqp, extra, la = _ln_bwd_fused(y, ln_w, ln_b, mean, rstd, None, dqpos,
                                                         dout, ctx.prev, cdtype, qp, period,
                                                         ctx.needs_input_grad[3])
            _wgrad(wg, extra, arena and la)
        else:
            k_linear_wgrad_group(wg)
            dy, dlw, dlb, dqp = _ln_bwd(y, ln_w, ln_b, mean, rstd, None, dqpos, dout, qp, period,
                                        ctx.needs_input_grad[3])
        return (dy, dlw, dlb, dqp, None, None, dmem_pos if l_mp else None,
                dmem if l_m else None, dw_in, db_in, dw_out, db_out) + (None,) * 9


# the FFN block's pre-norm LayerNorm backward reads the up-projection's data-gradient slabs
# directly (retr_layernorm_bwd_slabs: one slab-epilogue launch and the bf16 dn round trip
# fewer, bitwise the same; round 6)
LN_BWD_SLABS = True

# bf16 FFN blocks at d_model 256 as one fused launch per direction (csrc/ffn.hip: the hidden
# activation chunk goes from the first GEMM's accumulators into the second GEMM's LDS operand;
# same bits as the two-launch path).  Off by default: measured slower than linear_fwd +
# linear_fwd_splitk (profiles/r4_ffn_fused.txt: one 4-wave block per CU, 10 % MFMA busy)
FUSE_FFN = False
_FFN_SPLITS = {}


def _ffn_splits(M, C, F, cdtype):
    """F-split of the fused FFN kernels, 0 where the shape / dtype runs the unfused path."""
    if cdtype != torch.bfloat16 or not FUSE_FFN:
        return 0
    key = (M, C, F)
    s = _FFN_SPLITS.get(key)
    if s is None:
        s = _FFN_SPLITS[key] = int(_lib.load().retr_ffn_splits(M, C, F))
    return s


class _FFNBlock(torch.autograd.Function):
    """x_new = x + drop(W2 relu(W1 LN(x) + b1) + b2)  — FFResidual(feed_forward)
    (models/transformer_modules.py:6-11, 77-97) with its pre-norm inside the Function."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, eps, w1, b1, w2, b2, drop_res, cdtype, nxt=None):
        _lib.require_device(x)
        n, _, mean, rstd = _ln_fwd(x, ln_w, ln_b, eps, cdtype)
        res = x
        M, C = n.shape
        F = w1.shape[0]
        dev = n.device
        w1c, w2c = WEIGHTS.get(w1, cdtype), WEIGHTS.get(w2, cdtype)
        h = torch.empty(M, F, dtype=cdtype, device=dev)
        out = torch.empty(M, C, dtype=torch.float32, device=dev)
        splits = _ffn_splits(M, C, F, cdtype)
        if splits:
            seed = next_seed()
            ws = torch.empty(splits, M, C, dtype=torch.float32, device=dev)
            b1d, b2d = b1.detach().contiguous(), b2.detach().contiguous()
            call("retr_ffn_fwd", ptr(n), n.stride(0), ptr(w1c), ptr(b1d), ptr(w2c), ptr(b2d),
                 ptr(h), h.stride(0), ptr(res), res.stride(0), ptr(out), out.stride(0), M, C, F,
                 drop_res, seed, ptr(ws), splits, _st())
        else:
            k_linear_fwd(n, w1c, b1.detach(), h, relu=1)
            seed = next_seed()
            lnq = None
            if nxt is not None and FUSE_LN_NEXT and cdtype == torch.bfloat16:
                # the next norm's LayerNorm in this linear's epilogue (see _ln_take)
                g, bb, e2, pos, period, plain, with_pos = nxt
                ly = torch.empty(M, C, dtype=cdtype, device=dev) if plain else None
                ly2 = torch.empty(M, C, dtype=cdtype, device=dev) if with_pos else None
                mean2 = torch.empty(M, dtype=torch.float32, device=dev)
                rstd2 = torch.empty_like(mean2)
                lnq = (g, bb, e2, ly, ly2, pos, period, mean2, rstd2)
            k_linear_fwd(h, w2c, b2.detach(), out, res=res, drop_p=drop_res, seed=seed, ln=lnq)
            if lnq is not None:
                out._retr_ln = (_ln_key(g, bb, e2, pos, period, plain, with_pos, cdtype),
                                out._version, (ly, ly2, mean2, rstd2))
        ctx.splits = splits
        ctx.save_for_backward(n, h, w1, w2, x, ln_w, mean, rstd)
        ctx.gparams = (w1, b1, w2, b2)
        ctx.ln_b = ln_b
        ctx.cfg = (drop_res, seed, cdtype)
        ctx.prev = getattr(x, "_retr_drop", None)
        return _tag_drop(out, drop_res, seed)

    @staticmethod
    def backward(ctx, dout):
        n, h, w1, w2, x, ln_w, mean, rstd = ctx.saved_tensors
        drop_res, seed, cdtype = ctx.cfg
        M, C = n.shape
        F = h.shape[1]
        dev = n.device
        dout = dout.contiguous()
        w1t, w2t = WEIGHTS.get_t(w1, cdtype), WEIGHTS.get_t(w2, cdtype)
        fused = cdtype == torch.bfloat16 and FUSE_LN_BWD
        if fused:
            dbr = _take_dbr(dout, drop_res, seed, cdtype)
        else:
            dbr = torch.empty(M, C, dtype=cdtype, device=dev)
            k_dropout_apply(dout, dbr, drop_res, seed)
        (dw1, a0), (db1, a1), (dw2, a2), (db2, a3) = map(grad_buffer, ctx.gparams)
        arena = a0 and a1 and a2 and a3
        dh = torch.empty(M, F, dtype=cdtype, device=dev)
        dn = torch.empty(M, C, dtype=cdtype, device=dev)
        slabs = None
        if ctx.splits:
            # one fused launch: dh = [h > 0] dbr W2 (written for the weight gradients), dn = dh W1
            w1c, w2c = WEIGHTS.get(w1, cdtype), WEIGHTS.get(w2, cdtype)
            ws = torch.empty(ctx.splits, M, C, dtype=torch.float32, device=dev)
            call("retr_ffn_bwd_data", ptr(dbr), dbr.stride(0), ptr(w2c), ptr(h), h.stride(0),
                 ptr(w1c), ptr(dh), dh.stride(0), ptr(dn), dn.stride(0), M, C, F, ptr(ws),
                 ctx.splits, _st())
        else:
            k_linear_dgrad(dbr, w2t, dh, gate=h)
            sp = _splits(cdtype, M, C, F)
            if fused and LN_BWD_SLABS and sp > 1 and C in (256, 512):
                # the up-projection's data gradient as split-K slabs only, summed (in slice
                # order, rounded to bf16 as its epilogue would) by the LayerNorm backward
                sws = torch.empty(sp, M, C, dtype=torch.float32, device=dev)
                if isinstance(w1t, _TView):
                    w1p, w1tr = w1t.w, 0
                else:
                    w1p, w1tr = w1t, 1
                call("retr_linear_dgrad_slabs", dcode(cdtype), ptr(dh), dh.stride(0), ptr(w1p),
                     w1p.stride(0), M, F, C, w1tr, ptr(sws), sp, _st())
                slabs = (sws, sp)
            else:
                k_linear_dgrad(dh, w1t, dn)
        wg = [(dbr, h, dw2, db2, True), (dh, n, dw1, db1, True)]
        if fused:
            dx, dlw, dlb, _, extra, la = _ln_bwd_fused(x, ln_w, ctx.ln_b, mean, rstd,
                                                       dn if slabs is None else None, None,
                                                       dout, ctx.prev, cdtype, slabs=slabs)
            _wgrad(wg, extra, arena and la)
        else:
            k_linear_wgrad_group(wg)
            dx, dlw, dlb, _ = _ln_bwd(x, ln_w, ctx.ln_b, mean, rstd, dn, None, dout)
        return dx, dlw, dlb, None, dw1, db1, dw2, db2, None, None, None


def self_attn_block(res_mod, x, pos, period, B, L, kpm, causal, training, cdtype,
                    want_probs=False):
    """res_mod: SelfAttResidual container (.norm, .sublayer = nn.MultiheadAttention,
    .dropout); x: fp32 residual rows [B*L, C]; pos: position rows (table[row % period])."""
    sub = res_mod.sublayer
    return _SelfAttnBlock.apply(x, res_mod.norm.weight, res_mod.norm.bias, pos, period,
                                res_mod.norm.eps, sub.in_proj_weight, sub.in_proj_bias,
                                sub.out_proj.weight, sub.out_proj.bias, B, L, sub.num_heads, kpm,
                                causal, _drop_p(training, sub.dropout),
                                _drop_p(training, res_mod.dropout.p), cdtype, want_probs)


def cross_attn_block(res_mod, y, qpos, period, mem_pos, mem, B, Lq, Lk, kpm, training, cdtype,
                     want_probs=False):
    """res_mod: CrossAttResidual container; y: fp32 residual rows of the queries."""
    sub = res_mod.sublayer
    return _CrossAttnBlock.apply(y, res_mod.norm.weight, res_mod.norm.bias, qpos, period,
                                 res_mod.norm.eps, mem_pos, mem, sub.in_proj_weight,
                                 sub.in_proj_bias, sub.out_proj.weight, sub.out_proj.bias, B,
                                 Lq, Lk, sub.num_heads, kpm, _drop_p(training, sub.dropout),
                                 _drop_p(training, res_mod.dropout.p), cdtype, want_probs)


def ffn_block(res_mod, x, training, cdtype, next_norm=None):
    """res_mod: FFResidual container (.norm, .sublayer = Sequential(Linear, ReLU, Linear)).
    ``next_norm`` = (LayerNorm module, pos, period, plain, with_pos) of the LayerNorm that reads
    the output next (the following pre-norm block's or the stack's final norm): produced in the
    down-projection's epilogue (see _ln_take)."""
    seq = res_mod.sublayer
    nxt = None
    if next_norm is not None:
        nm, pos, period, plain, with_pos = next_norm
        nxt = (nm.weight, nm.bias, nm.eps, pos, period, plain, with_pos)
    return _FFNBlock.apply(x, res_mod.norm.weight, res_mod.norm.bias, res_mod.norm.eps,
                           seq[0].weight, seq[0].bias, seq[2].weight, seq[2].bias,
                           _drop_p(training, res_mod.dropout.p), cdtype, nxt)


# ---------------------------------------------------------------------------------------------
# decoder embeddings
# ---------------------------------------------------------------------------------------------

class _EmbedLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, caps, word, posw, gamma, beta, eps, drop_p, padding_idx, shared):
        B, T = caps.shape
        C = word.shape[1]
        if T > posw.shape[0]:
            raise RuntimeError(f"caption length {T} exceeds max_position_embeddings "
                               f"{posw.shape[0]}")
        dev = word.device
        caps = caps.contiguous()
        y = torch.empty(B * T, C, dtype=torch.float32, device=dev)
        mean = torch.empty(B * T, dtype=torch.float32, device=dev)
        rstd = torch.empty_like(mean)
        seed = next_seed()
        call("retr_embed_ln_fwd", ptr(caps), B, T, C, ptr(word), ptr(posw), ptr(gamma),
             ptr(beta), float(eps), drop_p, seed, ptr(y), ptr(mean), ptr(rstd), _st())
        ctx.save_for_backward(caps, word, posw, gamma, mean, rstd)
        ctx.gparams = (word, posw, gamma, beta)
        ctx.cfg = (eps, drop_p, seed, padding_idx)
        # the decoder blocks add their query-position gradients into one shared buffer of the
        # table (_shared_grad); the embedding's own position sum joins it, so autograd gets ONE
        # gradient for the parameter (adopted, never read) instead of two to add
        ctx.shared = bool(shared) and posw.requires_grad
        if ctx.shared:
            _share(posw)
        return y

    @staticmethod
    def backward(ctx, dy):
        caps, word, posw, gamma, mean, rstd = ctx.saved_tensors
        eps, drop_p, seed, padding_idx = ctx.cfg
        B, T = caps.shape
        C = word.shape[1]
        dev = word.device
        dy = dy.contiguous()
        wp, pp, gp, bp = ctx.gparams
        (dword, _), (dgamma, _), (dbeta, _) = map(grad_buffer, (wp, gp, bp))
        dposw, last = None, True
        if ctx.needs_input_grad[2] or ctx.shared:
            if ctx.shared:
                (dposw, _), _, last = _shared_grad(pp, lambda: grad_buffer(pp))
                # the decoder blocks' queued sums land first: (sum of blocks) + embedding, the
                # order of the per-block launches followed by autograd's add
                flush_pos(dposw.data_ptr())
            else:
                dposw, _ = grad_buffer(pp)
        M = B * T    # workspace: retr_embed_ln_bwd_workspace(B, T, C) bytes
        ws = torch.empty(M * C + 2 * C * ((M + 31) // 32), dtype=torch.float32, device=dev)
        call("retr_embed_ln_bwd", ptr(caps), B, T, C, ptr(word), ptr(posw), ptr(gamma),
             ptr(mean), ptr(rstd), ptr(dy), drop_p, seed, ptr(dword), ptr(dposw), ptr(dgamma),
             ptr(dbeta), -1 if padding_idx is None else int(padding_idx), ptr(ws), _st())
        if not (last and ctx.needs_input_grad[2]):
            dposw = None
        return None, dword, dposw, dgamma, dbeta, None, None, None, None


def embed_ln(emb, caps, training, shared=False):
    """emb: DecoderEmbeddings parameter container.  ``shared``: the position table's gradient
    is also accumulated by the blocks that read it as query positions in this pass
    (ConcatTransformer.decode, after begin_pass)."""
    p = _drop_p(training, emb.dropout.p)
    we = emb.word_embeddings
    return _EmbedLN.apply(caps, we.weight, emb.position_embeddings.weight, emb.LayerNorm.weight,
                          emb.LayerNorm.bias, emb.LayerNorm.eps, p, we.padding_idx,
                          shared and torch.is_grad_enabled())


# ---------------------------------------------------------------------------------------------
# plain linear (input_proj) and the MLP head
# ---------------------------------------------------------------------------------------------

class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, out_f32, dgate, cdtype):
        M, K = x.shape
        N = w.shape[0]
        wc = WEIGHTS.get(w, cdtype).view(N, -1)
        y = torch.empty(M, N, dtype=torch.float32 if out_f32 else cdtype, device=x.device)
        k_linear_fwd(x, wc, b.detach() if b is not None else None, y)
        ctx.save_for_backward(x, w, dgate)
        ctx.gparams = (w, b)
        ctx.cdtype = cdtype
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, dgate = ctx.saved_tensors
        cdtype = ctx.cdtype
        M, K = x.shape
        N = w.shape[0]
        dev = x.device
        if dy.dtype != cdtype or not dy.is_contiguous():
            dyc = torch.empty(M, N, dtype=cdtype, device=dev)
            k_dropout_apply(dy.float().contiguous(), dyc, 0.0, 0)
            dy = dyc
        dw, _ = grad_buffer(w)
        db = grad_buffer(ctx.gparams[1])[0] if ctx.has_b else None
        k_linear_wgrad(dy, x, dw.view(N, K), db, accumulate=True)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, dtype=cdtype, device=dev)
            k_linear_dgrad(dy, WEIGHTS.get_t(w, cdtype), dx, gate=dgate)
        return dx, dw, db, None, None, None


def linear(x, w, b, cdtype, out_f32=False, dgate=None):
    """y = x W^T + b.  ``dgate``: forward ReLU output feeding x; the data gradient is gated by
    ``dgate > 0`` inside the dgrad epilogue (fuses the producer's ReLU backward)."""
    return _Linear.apply(x, w, b, out_f32, dgate, cdtype)


def _round_up(n, m):
    return (n + m - 1) // m * m


class _MLPHead(torch.autograd.Function):
    """logits = L3(relu(L2(relu(L1 hs))))  with the vocabulary dim padded to a multiple of 64
    in memory; returns the [B, T, V] view."""

    @staticmethod
    def forward(ctx, hs, w1, b1, w2, b2, w3, b3, B, T, cdtype):
        M, C = hs.shape
        V = w3.shape[0]
        Vp = _round_up(V, 64)
        dev = hs.device
        w1c, w2c = WEIGHTS.get(w1, cdtype), WEIGHTS.get(w2, cdtype)
        w3c = WEIGHTS.get(w3, cdtype, rows=Vp)
        b3p = _pad_vec(b3, Vp)
        h1 = torch.empty(M, w1.shape[0], dtype=cdtype, device=dev)
        k_linear_fwd(hs, w1c, b1.detach(), h1, relu=1)
        h2 = torch.empty(M, w2.shape[0], dtype=cdtype, device=dev)
        k_linear_fwd(h1, w2c, b2.detach(), h2, relu=1)
        logits = torch.empty(M, Vp, dtype=cdtype, device=dev)
        k_linear_fwd(h2, w3c, b3p, logits)
        ctx.save_for_backward(hs, h1, h2, w1, w2, w3)
        ctx.gparams = (w1, b1, w2, b2, w3, b3)
        ctx.cfg = (B, T, V, Vp, cdtype)
        return logits[:, :V].view(B, T, V)

    @staticmethod
    def backward(ctx, dlog):
        hs, h1, h2, w1, w2, w3 = ctx.saved_tensors
        B, T, V, Vp, cdtype = ctx.cfg
        M, C = hs.shape
        dev = hs.device
        # fast path: the gradient is a view of a padded [M, Vp] compute-dtype buffer (from
        # cross_entropy); otherwise materialise one.
        if (dlog.dtype == cdtype and dlog.stride(2) == 1 and dlog.stride(1) == Vp
                and dlog.stride(0) == T * Vp):
            dl = dlog.as_strided((M, Vp), (Vp, 1))
        else:
            dl = torch.zeros(M, Vp, dtype=cdtype, device=dev)
            dl[:, :V] = dlog.reshape(M, V).to(cdtype)
        w1t, w2t = WEIGHTS.get_t(w1, cdtype), WEIGHTS.get_t(w2, cdtype)
        w3t = WEIGHTS.get_t(w3, cdtype, rows=Vp)
        bufs = list(map(grad_buffer, ctx.gparams))
        (dw1, _), (db1, _), (dw2, _), (db2, _), (dw3, _), (db3, _) = bufs
        # bf16 with every buffer in the optimizer arena: the three weight gradients (+ biases,
        # as the batch's all-ones MFMA instead of a column-sum launch over the 125 MB dlogits)
        # join the deferred batch that the transformer blocks' backward fills (one launch at the
        # transformer input fence; see _wgrad)
        defer = (HEAD_WGRAD_DEFER and WGRAD_DEFER and cdtype == torch.bfloat16
                 and all(a for _, a in bufs))
        ov = _Overlap(OVERLAP["transformer"])
        if defer:
            _wgrad([(dl, h2, dw3, db3, True)], (), True)     # N = V rows of the padded dl
        else:
            with ov.side():
                k_linear_wgrad(dl, h2, dw3, db3, accumulate=True)
        dh2 = torch.empty_like(h2)
        k_linear_dgrad(dl, w3t, dh2, gate=h2)
        if defer:
            _wgrad([(dh2, h1, dw2, db2, True)], (), True)
        else:
            with ov.side():
                k_linear_wgrad(dh2, h1, dw2, db2, accumulate=True)
        dh1 = torch.empty_like(h1)
        k_linear_dgrad(dh2, w2t, dh1, gate=h1)
        if defer:
            _wgrad([(dh1, hs, dw1, db1, True)], (), True)
        else:
            with ov.side():
                k_linear_wgrad(dh1, hs, dw1, db1, accumulate=True)
        dhs = torch.empty_like(hs)
        k_linear_dgrad(dh1, w1t, dhs)
        ov.join()
        return dhs, dw1, db1, dw2, db2, dw3, db3, None, None, None


def mlp_head(mlp, hs, B, T, cdtype):
    l1, l2, l3 = mlp.layers
    return _MLPHead.apply(hs, l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias, B, T,
                          cdtype)


# ---------------------------------------------------------------------------------------------
# cross entropy (engine.py:71: criterion(outputs.permute(0, 2, 1), caps[:, 1:]))
# ---------------------------------------------------------------------------------------------

FUSED_CE = True   # bf16 training: loss and dlogits from one pass (tests / A/B switch it off)
_TRAIN_STEP = 0   # > 0 inside train_step_scope(): a backward pass is about to follow


class train_step_scope:
    """Marks a forward whose loss will be back-propagated right away (engine.forward_backward,
    engine.train_one_epoch).  Only there does the cross-entropy compute dlogits in its forward
    pass (retr_ce_fwd_bwd): a loss computed with grad enabled for logging, or a step that fails
    before backward, then costs no extra [M, Vp] buffer or HBM pass."""

    def __enter__(self):
        global _TRAIN_STEP
        _TRAIN_STEP += 1
        return self

    def __exit__(self, *exc):
        global _TRAIN_STEP
        _TRAIN_STEP -= 1
        return False


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target):
        # x: [B, V, T] (permuted view of [B, T, V] logits whose rows may be padded)
        _lib.require_device(x, target)
        B, V, T = x.shape
        if x.stride(1) == 1 and x.stride(0) == T * x.stride(2):
            base, ld = x, x.stride(2)
        else:
            base = x.permute(0, 2, 1).contiguous()
            ld = V
        M = B * T
        dev = x.device
        tgt = target.reshape(M).contiguous()
        lse = torch.empty(M, dtype=torch.float32, device=dev)
        rows = torch.empty(M, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        Vp = _round_up(V, 64)
        ctx.dl = None
        if (ctx.needs_input_grad[0] and base.dtype == torch.bfloat16 and ld % 8 == 0
                and Vp <= 32768 and FUSED_CE and _TRAIN_STEP > 0):
            # training: the gradient for dloss = 1 comes out of the same pass over the logits
            # (retr_ce_fwd_bwd); backward only rewrites it if dloss != 1
            ctx.dl = torch.empty(M, Vp, dtype=base.dtype, device=dev)
            call("retr_ce_fwd_bwd", dcode(base.dtype), ptr(base), ld, M, V, ptr(tgt), ptr(lse),
                 ptr(rows), ptr(loss), 1.0 / M, ptr(ctx.dl), Vp, _st())
        else:
            call("retr_ce_fwd", dcode(base.dtype), ptr(base), ld, M, V, ptr(tgt), ptr(lse),
                 ptr(rows), ptr(loss), _st())
        ctx.save_for_backward(base, tgt, lse)
        ctx.cfg = (B, V, T, ld)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        base, tgt, lse = ctx.saved_tensors
        B, V, T, ld = ctx.cfg
        M = B * T
        Vp = _round_up(V, 64)
        dloss = dloss.reshape(1).float().contiguous()
        dl = ctx.dl
        ctx.dl = None
        if dl is not None:
            call("retr_ce_bwd_rescale", dcode(base.dtype), ptr(base), ld, M, V, ptr(tgt),
                 ptr(lse), ptr(dloss), 1.0 / M, ptr(dl), Vp, _st())
        else:
            dl = torch.empty(M, Vp, dtype=base.dtype, device=base.device)
            call("retr_ce_bwd", dcode(base.dtype), ptr(base), ld, M, V, ptr(tgt), ptr(lse),
                 ptr(dloss), 1.0 / M, ptr(dl), Vp, _st())
        return dl[:, :V].view(B, T, V).permute(0, 2, 1), None


def cross_entropy(x, target):
    return _CrossEntropy.apply(x, target)


def argmax_rows(x2d):
    """First-index argmax over the last dim of a [M, V] (row-strided) tensor."""
    M, V = x2d.shape
    out = torch.empty(M, dtype=torch.long, device=x2d.device)
    call("retr_argmax_rows", dcode(x2d.dtype), ptr(x2d), x2d.stride(0), M, V, ptr(out), _st())
    return out


# ---------------------------------------------------------------------------------------------
# encoder output without a final LayerNorm (pre_norm=False) and learned position embeddings
# ---------------------------------------------------------------------------------------------

class _AddPos(torch.autograd.Function):
    """(cast(x), cast(x + pos[row % period])): memory and memory+pos for the decoder when the
    encoder has no final LayerNorm (models/ConcatTransformer.py:24, :105-106 with
    normalize_before=False; the cross-attention keys add ``pos`` at
    transformer_modules.py:61-62)."""

    @staticmethod
    def forward(ctx, x, pos, period, cdtype):
        _lib.require_device(x)
        M, C = x.shape
        y = torch.empty(M, C, dtype=cdtype, device=x.device)
        y2 = torch.empty_like(y)
        posd = pos.detach().contiguous()
        call("retr_add_pos_fwd", dcode(cdtype), ptr(x), x.stride(0), M, C, ptr(posd), int(period),
             ptr(y), ptr(y2), C, _st())
        ctx.cfg = (M, C, period, tuple(pos.shape))
        return y, y2

    @staticmethod
    def backward(ctx, dy, dy2):
        M, C, period, pshape = ctx.cfg
        ref = dy if dy is not None else dy2
        dev = ref.device
        dy = dy.contiguous() if dy is not None else None
        dy2 = dy2.contiguous() if dy2 is not None else None
        if dy is not None and dy2 is not None and dy.dtype != dy2.dtype:
            dy2 = dy2.to(dy.dtype)
        dx = torch.empty(M, C, dtype=torch.float32, device=dev)
        call("retr_sum2", dcode(ref.dtype), ptr(dy), ptr(dy2), M * C, ptr(dx), _st())
        dpos = None
        if ctx.needs_input_grad[1] and dy2 is not None:
            dpos = torch.empty(pshape, dtype=torch.float32, device=dev)
            call("retr_pos_grad_set", dcode(dy2.dtype), ptr(dy2), C, M, C, period, ptr(dpos),
                 _st())
        return dx, dpos, None, None


def add_pos(x, pos, period, cdtype):
    return _AddPos.apply(x, pos, period, cdtype)


class _LearnedPos(torch.autograd.Function):
    """PositionalEmbedding.forward (models/position_encoding.py:50-63): the [S, C] table
    LayerNorm(pos_embed[0:S]) repeated over the batch and dropped out per (b, s, c) (dropout
    after the repeat, so every sample has its own mask).  Returns batch-major rows
    [B*S, C] fp32 (consumed by the fused LayerNorm + position kernels with period B*S)."""

    @staticmethod
    def forward(ctx, weight, gamma, beta, B, S, eps, drop_p):
        _lib.require_device(weight)
        C = weight.shape[1]
        dev = weight.device
        if S > weight.shape[0]:
            raise RuntimeError(f"index out of range: position {S - 1} >= num_embeddings "
                               f"{weight.shape[0]}")
        tab = torch.empty(S, C, dtype=torch.float32, device=dev)
        mean = torch.empty(S, dtype=torch.float32, device=dev)
        rstd = torch.empty_like(mean)
        wd = weight.detach()
        call("retr_layernorm_fwd", F32, ptr(wd), wd.stride(0), ptr(gamma), ptr(beta), float(eps),
             S, C, ptr(tab), C, None, None, 1, ptr(mean), ptr(rstd), _st())
        rep = tab.repeat(B, 1)
        seed = next_seed()
        if drop_p > 0:
            call("retr_dropout_apply", F32, ptr(rep), C, ptr(rep), C, B * S, C, float(drop_p),
                 seed, _st())
        ctx.save_for_backward(weight, gamma, mean, rstd)
        ctx.beta = beta
        ctx.cfg = (B, S, C, drop_p, seed)
        return rep

    @staticmethod
    def backward(ctx, dout):
        weight, gamma, mean, rstd = ctx.saved_tensors
        B, S, C, drop_p, seed = ctx.cfg
        dev = weight.device
        d = dout.float().contiguous()
        if drop_p > 0:
            dd = torch.empty_like(d)
            call("retr_dropout_apply", F32, ptr(d), C, ptr(dd), C, B * S, C, float(drop_p), seed,
                 _st())
            d = dd
        dtab = torch.empty(S, C, dtype=torch.float32, device=dev)
        call("retr_pos_grad_set", F32, ptr(d), C, B * S, C, S, ptr(dtab), _st())
        dw, _ = grad_buffer(weight)
        dgamma, _ = grad_buffer(gamma)
        dbeta, _ = grad_buffer(ctx.beta)
        wd = weight.detach()
        # rows 0..S-1 of the (zeroed) embedding gradient are written directly; rows >= S get
        # no gradient, as from nn.Embedding with ids arange(S)
        call("retr_layernorm_bwd", F32, ptr(dtab), None, C, ptr(wd), wd.stride(0), ptr(gamma),
             ptr(mean), ptr(rstd), S, C, ptr(dw), dw.stride(0), None, ptr(dgamma), ptr(dbeta),
             ptr(ln_workspace(S, C, dev)), _st())
        return dw, dgamma, dbeta, None, None, None, None


def learned_pos(pe_module, B, S, training):
    """pe_module: PositionalEmbedding container (.pos_embed, .LayerNorm, .dropout)."""
    return _LearnedPos.apply(pe_module.pos_embed.weight, pe_module.LayerNorm.weight,
                             pe_module.LayerNorm.bias, B, S, pe_module.LayerNorm.eps,
                             _drop_p(training, pe_module.dropout.p))
