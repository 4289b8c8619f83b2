"""ResNet body executor: NHWC implicit-GEMM convolutions with FrozenBatchNorm folded into the
weights, fused bias/residual/ReLU epilogues, and a hand-scheduled backward.

Replaces the torchvision conv stack that ``models/backbone.py:65,69`` runs through
``IntermediateLayerGetter`` (return layer4 only), with FrozenBatchNorm2d
(``models/backbone.py:41-51``: scale = w * rsqrt(rv + 1e-5), bias = b - rm * scale) folded:
``conv(x, W) * scale + bias == conv(x, W * scale) + bias``.

Backward (only blocks whose parameters require grad — the reference freezes stem + layer1,
``models/backbone.py:58-60``):
  G3 = dOut * (out > 0)                          (gate fused into the consumer's dgrad epilogue)
  dW3 = wgrad(G3, h2) * s3 ;  G2 = dgrad(G3, W3eff) * (h2 > 0)
  dW2 = wgrad(G2, h1) * s2 ;  G1 = dgrad(G2, W2eff) * (h1 > 0)
  dW1 = wgrad(G1, x)  * s1 ;  dWds = wgrad(G3, x) * sds
  G3_prev = (dgrad(G1, W1eff) + [G3 | dgrad(G3, Wdseff)]) * (x > 0)
"""
import os

import torch

from . import _lib
from ._lib import call, ptr
from .optim import grad_buffer
from .ops import dcode, _st


class ConvSpec:
    __slots__ = ("conv", "bn", "k", "s", "p", "d", "cin", "cout", "cp", "pack")

    def __init__(self, conv, bn, stride=1, padding=0, dilation=1):
        self.conv, self.bn = conv, bn
        self.k = conv.weight.shape[2]
        self.s, self.p, self.d = stride, padding, dilation
        self.cout, self.cin = conv.weight.shape[0], conv.weight.shape[1]
        self.cp = max(8, (self.cin + 7) // 8 * 8)
        self.pack = None            # (version key, packed tensors): _PackCache

    def out_hw(self, h, w):
        oh = (h + 2 * self.p - self.d * (self.k - 1) - 1) // self.s + 1
        ow = (w + 2 * self.p - self.d * (self.k - 1) - 1) // self.s + 1
        return oh, ow


class BlockSpec:
    __slots__ = ("kind", "convs", "ds", "name")

    def __init__(self, name, kind, convs, ds):
        self.name, self.kind, self.convs, self.ds = name, kind, convs, ds

    def params(self):
        ps = [c.conv.weight for c in self.convs]
        if self.ds is not None:
            ps.append(self.ds.conv.weight)
        return ps

    def trainable(self):
        return any(p.requires_grad for p in self.params())


def build_plan(body):
    """body: the IntermediateLayerGetter-equivalent ModuleDict (conv1, bn1, layer1..layer4)."""
    stem = ConvSpec(body.conv1, body.bn1, 2, 3, 1)
    blocks = []
    for li in range(1, 5):
        layer = getattr(body, f"layer{li}")
        for bi, blk in enumerate(layer):
            ds = None
            if blk.downsample is not None:
                ds = ConvSpec(blk.downsample[0], blk.downsample[1], blk.downsample[0].stride[0])
            if hasattr(blk, "conv3"):
                c2 = blk.conv2
                convs = [ConvSpec(blk.conv1, blk.bn1),
                         ConvSpec(c2, blk.bn2, c2.stride[0], c2.padding[0], c2.dilation[0]),
                         ConvSpec(blk.conv3, blk.bn3)]
                kind = "bottleneck"
            else:
                c1 = blk.conv1
                convs = [ConvSpec(c1, blk.bn1, c1.stride[0], c1.padding[0], c1.dilation[0]),
                         ConvSpec(blk.conv2, blk.bn2, 1, 1, 1)]
                kind = "basic"
            blocks.append(BlockSpec(f"layer{li}.{bi}", kind, convs, ds))
    return stem, blocks


class _PackCache:
    """Folded compute-dtype weights per conv, refreshed when the weight or a BN buffer changes.
    The entry lives on the ConvSpec itself (it dies with its model): a dict keyed by id(spec)
    could hand a new model, whose spec reuses a dead one's id and whose tensors reuse its
    addresses, the dead model's packed weights."""

    def get(self, spec, dtype):
        w = spec.conv.weight
        bn = spec.bn
        ver = (w._version, w.data_ptr(), dtype) + tuple(
            (b._version, b.data_ptr()) for b in (bn.weight, bn.bias, bn.running_mean,
                                                 bn.running_var))
        ent = spec.pack
        if ent is not None and ent[0] == ver:
            return ent[1]
        co, ci, k = spec.cout, spec.cin, spec.k
        wp = torch.empty(co, k, k, spec.cp, dtype=dtype, device=w.device)
        wt = torch.empty(spec.cp, k, k, co, dtype=dtype, device=w.device)
        bias = torch.empty(co, dtype=torch.float32, device=w.device)
        scale = torch.empty(co, dtype=torch.float32, device=w.device)
        wd = w.detach().contiguous()
        call("retr_conv_pack", dcode(dtype), ptr(wd), ptr(bn.weight), ptr(bn.bias),
             ptr(bn.running_mean), ptr(bn.running_var), None, co, ci, k, k, spec.cp, ptr(wp),
             ptr(wt), ptr(bias), ptr(scale), _st())
        out = (wp, wt, bias, scale)
        spec.pack = (ver, out)
        return out


    def prepare(self, specs, dtype):
        """Pack every stale conv of ``specs`` in one grouped launch (retr_conv_pack_group)."""
        todo = []
        for spec in specs:
            w, bn = spec.conv.weight, spec.bn
            ver = (w._version, w.data_ptr(), dtype) + tuple(
                (b._version, b.data_ptr()) for b in (bn.weight, bn.bias, bn.running_mean,
                                                     bn.running_var))
            ent = spec.pack
            if ent is None or ent[0] != ver:
                todo.append((spec, ver))
        if not todo:
            return
        arr = (_lib.ConvPackDesc * len(todo))()
        keep = []
        for i, (spec, ver) in enumerate(todo):
            w, bn = spec.conv.weight, spec.bn
            co, ci, k = spec.cout, spec.cin, spec.k
            dev = w.device
            wp = torch.empty(co, k, k, spec.cp, dtype=dtype, device=dev)
            wt = torch.empty(spec.cp, k, k, co, dtype=dtype, device=dev)
            bias = torch.empty(co, dtype=torch.float32, device=dev)
            scale = torch.empty(co, dtype=torch.float32, device=dev)
            wd = w.detach().contiguous()
            keep.append(wd)
            d = arr[i]
            d.w, d.bn_w, d.bn_b = ptr(wd), ptr(bn.weight), ptr(bn.bias)
            d.bn_rm, d.bn_rv, d.conv_bias = ptr(bn.running_mean), ptr(bn.running_var), None
            d.w_out, d.wt_out, d.bias_out, d.scale_out = ptr(wp), ptr(wt), ptr(bias), ptr(scale)
            d.Co, d.Ci, d.KH, d.KW, d.Cp = co, ci, k, k, spec.cp
            spec.pack = (ver, (wp, wt, bias, scale))
        call("retr_conv_pack_group", dcode(dtype), len(todo), arr, _st())


PACKS = _PackCache()


def _conv_fwd(spec, x, shape, relu, residual=None):
    n, h, w, c = shape
    oh, ow = spec.out_hw(h, w)
    wp, _, bias, _ = PACKS.get(spec, x.dtype)
    y = torch.empty(n, oh, ow, spec.cout, dtype=x.dtype, device=x.device)
    call("retr_conv2d_fwd", dcode(x.dtype), ptr(x), n, h, w, c, ptr(wp), ptr(bias), ptr(residual),
         ptr(y), spec.cout, spec.k, spec.k, spec.s, spec.p, spec.d, int(relu), _st())
    return y, (n, oh, ow, spec.cout)


# first blocks' input gradient: the downsample's data gradient accumulated in place onto conv1's
# gated one (round 6; False: round 5's temporary + elementwise fill of the tap-less phases)
DS_DGRAD_INPLACE = True


def _conv_dgrad(spec, g, in_shape, addend=None, gate=None, out=None):
    n, h, w, c = in_shape
    _, wt, _, _ = PACKS.get(spec, g.dtype)
    dx = out if out is not None else torch.empty(n, h, w, c, dtype=g.dtype, device=g.device)
    call("retr_conv2d_dgrad", dcode(g.dtype), ptr(g), n, h, w, c, ptr(wt), ptr(dx), spec.cout,
         spec.k, spec.k, spec.s, spec.p, spec.d, ptr(addend), ptr(gate), _st())
    return dx


def wgrad_splits(dtype, n, h, w, c, spec):
    """Number of pixel-reduction slices (partial slabs) retr_conv2d_wgrad writes."""
    return int(_lib.load().retr_conv2d_wgrad_splits(dcode(dtype), n, h, w, c, spec.cout, spec.k,
                                                     spec.k, spec.s, spec.p, spec.d))


def _conv_wgrad(spec, g, x, in_shape):
    n, h, w, c = in_shape
    _, _, _, scale = PACKS.get(spec, g.dtype)
    splits = wgrad_splits(g.dtype, n, h, w, c, spec)
    ws = torch.empty(splits, spec.cout, spec.k * spec.k * c, dtype=torch.float32,
                     device=g.device)
    call("retr_conv2d_wgrad", dcode(g.dtype), ptr(g), ptr(x), n, h, w, c, ptr(ws), spec.cout,
         spec.k, spec.k, spec.s, spec.p, spec.d, _st())
    grad, _ = grad_buffer(spec.conv.weight)     # sole writer: overwrite mode below
    call("retr_conv_wgrad_unpack", ptr(ws), ptr(scale), ptr(grad), spec.cout, spec.cin, c, spec.k,
         spec.k, 0, splits, _st())
    return grad


# The bf16 backbone backward queues every conv weight gradient and runs them as one grouped
# launch per loader kind at the end (retr_conv2d_wgrad_group): one K-slice length over all
# convs instead of each conv's own split-K plan (which had to fill 256 CUs from 9-144 tiles),
# ~5x fewer fp32 slab bytes written and re-read by the unpacks.
CONV_WGRAD_GROUP = True
CONV_WGRAD_STATS = {"grouped": 0, "single": 0}


def _conv_wgrad_group(items, grads):
    """items: (spec, G, x, in_shape) of every conv weight gradient of one backward."""
    n = len(items)
    arr = (_lib.ConvWgradDesc * n)()
    for i, (spec, G, x, shape) in enumerate(items):
        nb, h, w, c = shape
        d = arr[i]
        d.dy, d.x = ptr(G), ptr(x)
        d.Nb, d.H, d.W, d.C, d.Co = nb, h, w, c, spec.cout
        d.KH = d.KW = spec.k
        d.stride, d.pad, d.dil = spec.s, spec.p, spec.d
    G0 = items[0][1]
    call("retr_conv2d_wgrad_group_plan", dcode(G0.dtype), n, arr)
    slabs = []
    for i, (spec, G, x, shape) in enumerate(items):
        if arr[i].kind < 0:
            grads[spec.conv.weight] = _conv_wgrad(spec, G, x, shape)
            CONV_WGRAD_STATS["single"] += 1
            slabs.append(None)
            continue
        c = shape[3]
        ws = torch.empty(arr[i].splits, spec.cout, spec.k * spec.k * c, dtype=torch.float32,
                         device=G.device)
        arr[i].ws = ptr(ws)
        slabs.append(ws)
    if any(t is not None for t in slabs):
        nbytes = int(_lib.load().retr_conv2d_wgrad_group_table_bytes(n)) + 512
        table = torch.empty(nbytes, dtype=torch.uint8, device=G0.device)
        call("retr_conv2d_wgrad_group", dcode(G0.dtype), n, arr, ptr(table), nbytes, _st())
    jobs = [i for i in range(n) if slabs[i] is not None]
    if not jobs:
        return
    ua = (_lib.ConvUnpackDesc * len(jobs))()
    for j, i in enumerate(jobs):
        spec, G, x, shape = items[i]
        _, _, _, scale = PACKS.get(spec, G.dtype)
        grad, _ = grad_buffer(spec.conv.weight)     # sole writer: overwrite mode
        u = ua[j]
        u.ws, u.scale, u.grad = ptr(slabs[i]), ptr(scale), ptr(grad)
        u.Co, u.Ci, u.Cp, u.KH, u.KW = spec.cout, spec.cin, shape[3], spec.k, spec.k
        u.splits, u.accumulate = arr[i].splits, 0
        grads[spec.conv.weight] = grad
        CONV_WGRAD_STATS["grouped"] += 1
    if all(ua[j].Ci % 4 == 0 for j in range(len(jobs))):
        nb = int(_lib.load().retr_conv_wgrad_unpack_group_table_bytes(len(jobs)))
        utab = torch.empty((nb + 15) // 16 * 16, dtype=torch.uint8, device=G0.device)
        call("retr_conv_wgrad_unpack_group", len(jobs), ua, ptr(utab), utab.numel(), _st())
        return
    for j in range(len(jobs)):                   # channel counts off the 4-wide chunks
        u = ua[j]
        call("retr_conv_wgrad_unpack", u.ws, u.scale, u.grad, u.Co, u.Ci, u.Cp, u.KH, u.KW, 0,
             u.splits, _st())


def _conv_tail_cat(runner, blk, h2, s2, x, xshape):
    """relu(conv3(h2) + downsample(x)) as one 1x1 conv over the channel concatenation
    (BackboneRunner.cat_tail); weights [W3eff | Wdseff] and bias b3 + bds cached per pack."""
    c3, ds = blk.convs[2], blk.ds
    wcat, bcat = _cat_weights(runner, blk, h2.dtype)
    n, oh, ow, c1 = s2
    y = torch.empty(n, oh, ow, c3.cout, dtype=h2.dtype, device=h2.device)
    call("retr_conv1x1_fwd_cat", dcode(h2.dtype), ptr(h2), c1, ptr(x), xshape[3], n, oh, ow,
         xshape[1], xshape[2], ds.s, ptr(wcat), ptr(bcat), ptr(y), c3.cout, 1, _st())
    runner.cat_used.append(blk.name)
    return y, (n, oh, ow, c3.cout)


def _cat_weights(runner, blk, dtype):
    """[W3eff | Wdseff] and b3 + bds of a block with a 1x1 downsample, cached per pack."""
    c3, ds = blk.convs[2], blk.ds
    wp3, _, b3, _ = PACKS.get(c3, dtype)
    wpd, _, bd, _ = PACKS.get(ds, dtype)
    ent = runner._cat_w.get(blk.name)
    if ent is None or ent[0] is not wp3 or ent[1] is not wpd:
        _prepare_cats(runner, dtype, [blk])
        ent = runner._cat_w[blk.name]
    return ent[2], ent[3]


def _prepare_cats(runner, dtype, blocks=None):
    """Refresh the [W3eff | Wdseff] / b3 + bds operands of every stale fused-tail block in one
    retr_cat_rows_group launch (bf16; after PACKS.prepare repacked the weights of the step)."""
    if dtype != torch.bfloat16 or not runner.use_cat:
        return
    todo = []
    for blk in (blocks if blocks is not None else runner.blocks):
        if blk.ds is None or blk.kind != "bottleneck":
            continue
        c3, ds = blk.convs[2], blk.ds
        wp3, _, b3, _ = PACKS.get(c3, dtype)
        wpd, _, bd, _ = PACKS.get(ds, dtype)
        ent = runner._cat_w.get(blk.name)
        if ent is not None and ent[0] is wp3 and ent[1] is wpd:
            continue
        ka, kb = wp3[0].numel(), wpd[0].numel()
        if ent is not None and ent[2].shape == (c3.cout, ka + kb):
            wcat, bcat = ent[2], ent[3]            # same shapes: refresh in place
        else:
            wcat = torch.empty(c3.cout, ka + kb, dtype=dtype, device=wp3.device)
            bcat = torch.empty(c3.cout, dtype=torch.float32, device=wp3.device)
        todo.append((blk, wp3, wpd, b3, bd, wcat, bcat, ka, kb))
    for i in range(0, len(todo), 8):
        chunk = todo[i:i + 8]
        arr = (_lib.CatRowsDesc * len(chunk))()
        for j, (blk, wp3, wpd, b3, bd, wcat, bcat, ka, kb) in enumerate(chunk):
            d = arr[j]
            d.a, d.b, d.dst = ptr(wp3), ptr(wpd), ptr(wcat)
            d.bias_a, d.bias_b, d.bias_dst = ptr(b3), ptr(bd), ptr(bcat)
            d.rows, d.ka, d.kb = wcat.shape[0], ka, kb
            runner._cat_w[blk.name] = (wp3, wpd, wcat, bcat)
        call("retr_cat_rows_group", len(chunk), arr, _st())


def _bottleneck_fused(runner, blk, x, xshape):
    """The whole stride-1 bottleneck in one launch (retr_bottleneck_s1_fwd): h1 / h2 stay in
    LDS, x is read once.  Only for blocks whose activations backward never needs (the frozen
    layer1, models/backbone.py:58-60)."""
    c1, c2, c3 = blk.convs
    n, h, w, cin = xshape
    wp1, _, b1, _ = PACKS.get(c1, x.dtype)
    wp2, _, b2, _ = PACKS.get(c2, x.dtype)
    if blk.ds is not None:
        w3, b3 = _cat_weights(runner, blk, x.dtype)
    else:
        w3, _, b3, _ = PACKS.get(c3, x.dtype)
    y = torch.empty(n, h, w, c3.cout, dtype=x.dtype, device=x.device)
    call("retr_bottleneck_s1_fwd", dcode(x.dtype), ptr(x), n, h, w, cin, ptr(wp1), ptr(b1),
         ptr(wp2), ptr(b2), ptr(w3), ptr(b3), int(blk.ds is not None), ptr(y), _st())
    runner.fused_used.append(blk.name)
    return y, (n, h, w, c3.cout)


def _stem_s2d(runner, img):
    """bf16 stem as a space-to-depth conv: the 3-channel image becomes [N, H/2, W/2, 16]
    (2x2 pixel blocks, 12 channels + 4 zero), the 7x7 stride-2 pad-3 kernel a 4x4 stride-1 pad-2
    one (retr_stem_s2d_weights) -- the same bf16 operands and products as torchvision's conv1
    (models/backbone.py:85-95), K = 256 instead of 392 and half the input bytes."""
    stem = runner.stem
    N, C, H, W = img.shape
    wp, _, bias, _ = PACKS.get(stem, runner.cdtype)
    if runner._s2d_w is None or runner._s2d_w[0] is not wp:
        w2 = torch.empty(stem.cout, 4, 4, 16, dtype=runner.cdtype, device=img.device)
        call("retr_stem_s2d_weights", ptr(wp), ptr(w2), stem.cout, stem.cp, _st())
        runner._s2d_w = (wp, w2)
    w2 = runner._s2d_w[1]
    h2, w2_ = H // 2, W // 2
    x = torch.empty(N, h2, w2_, 16, dtype=runner.cdtype, device=img.device)
    call("retr_nchw_to_s2d16", ptr(img), ptr(x), N, C, H, W, _st())
    if runner.stem_pool and stem.cout == 64:
        # conv + bias + ReLU + MaxPool(3, 2, 1) in one launch (csrc/stem.hip): the stem is
        # frozen (models/backbone.py:58-60), so its conv output is never needed again
        ph, pw = (h2 - 1) // 2 + 1, (w2_ - 1) // 2 + 1
        y = torch.empty(N, ph, pw, stem.cout, dtype=runner.cdtype, device=img.device)
        call("retr_stem_pool_fwd", dcode(runner.cdtype), ptr(x), N, h2, w2_, ptr(w2), ptr(bias),
             ptr(y), stem.cout, _st())
        return y, (N, ph, pw, stem.cout), True
    y = torch.empty(N, h2, w2_, stem.cout, dtype=runner.cdtype, device=img.device)
    call("retr_conv2d_fwd_out", dcode(runner.cdtype), ptr(x), N, h2, w2_, 16, ptr(w2), ptr(bias),
         None, ptr(y), stem.cout, 4, 4, 1, 2, 1, h2, w2_, 1, _st())
    return y, (N, h2, w2_, stem.cout), False


class _Backbone(torch.autograd.Function):
    @staticmethod
    def forward(ctx, images, runner, *weights):
        stem, blocks, cdtype = runner.stem, runner.blocks, runner.cdtype
        _lib.require_device(images)
        PACKS.prepare(runner.specs, cdtype)      # every stale conv packed in one launch
        _prepare_cats(runner, cdtype)            # and every fused tail's [W3 | Wds] in one more
        N, C, H, W = images.shape
        img = images.detach().float().contiguous()
        pooled = False
        if runner.s2d_stem(C, H, W):
            s, sh, pooled = _stem_s2d(runner, img)
        else:
            x = torch.empty(N, H, W, stem.cp, dtype=cdtype, device=images.device)
            call("retr_nchw_to_nhwc", dcode(cdtype), ptr(img), ptr(x), N, C, H, W, stem.cp, _st())
            s, sh = _conv_fwd(stem, x, (N, H, W, stem.cp), relu=True)
        if pooled:
            x, shape = s, sh
        else:
            ph, pw = (sh[1] + 2 - 3) // 2 + 1, (sh[2] + 2 - 3) // 2 + 1
            x = torch.empty(N, ph, pw, sh[3], dtype=cdtype, device=images.device)
            call("retr_maxpool3x3s2", dcode(cdtype), ptr(s), ptr(x), N, sh[1], sh[2], sh[3], ph,
                 pw, _st())
            shape = (N, ph, pw, sh[3])
        del s
        saved = []
        runner.cat_used = []
        runner.fused_used = []
        grad_on = runner.save
        for blk in blocks:
            inp, ishape = x, shape
            keep = grad_on and blk.trainable()
            if not keep and runner.fused_block(blk, ishape):
                x, shape = _bottleneck_fused(runner, blk, inp, ishape)
                continue
            if blk.kind == "bottleneck":
                c1, c2, c3 = blk.convs
                h1, s1 = _conv_fwd(c1, inp, ishape, True)
                h2, s2 = _conv_fwd(c2, h1, s1, True)
                if runner.cat_tail(blk, ishape, s2):
                    out, oshape = _conv_tail_cat(runner, blk, h2, s2, inp, ishape)
                else:
                    idt = _conv_fwd(blk.ds, inp, ishape, False)[0] if blk.ds is not None else inp
                    out, oshape = _conv_fwd(c3, h2, s2, True, residual=idt)
                acts = (inp, ishape, h1, s1, h2, s2)
            else:
                c1, c2 = blk.convs
                h1, s1 = _conv_fwd(c1, inp, ishape, True)
                idt = _conv_fwd(blk.ds, inp, ishape, False)[0] if blk.ds is not None else inp
                out, oshape = _conv_fwd(c2, h1, s1, True, residual=idt)
                acts = (inp, ishape, h1, s1, None, None)
            if keep:
                saved.append((blk, acts))
            x, shape = out, oshape
        ctx.runner = runner
        ctx.saved_acts = saved
        ctx.n_weights = len(weights)
        ctx.out_shape = shape
        return x

    @staticmethod
    def backward(ctx, g):
        # The data-gradient chain runs on the current stream; every weight gradient only needs
        # its conv's output gradient and input, so it runs on the side stream (ops._Overlap)
        # concurrently with the rest of the chain.  Tensors the side work reads stay referenced
        # in ``keep`` until the final join, so the caching allocator cannot hand their memory
        # to the chain while the side stream still reads it.
        from .ops import OVERLAP, _Overlap
        runner = ctx.runner
        grads = {}
        g = g.contiguous()
        saved = ctx.saved_acts
        ov = _Overlap(OVERLAP["backbone"])
        keep = []
        group = CONV_WGRAD_GROUP and g.dtype == torch.bfloat16 and not OVERLAP["backbone"]
        pending = []

        def wgrad(spec, G, x, shape):
            if group:
                pending.append((spec, G, x, shape))
                return
            keep.extend((G, x))
            with ov.side():
                grads[spec.conv.weight] = _conv_wgrad(spec, G, x, shape)

        for idx in range(len(saved) - 1, -1, -1):
            blk, (inp, ishape, h1, s1, h2, s2) = saved[idx]
            need_dx = idx > 0 and saved[idx - 1][0] is runner.blocks[runner.blocks.index(blk) - 1]
            G3 = g
            if blk.kind == "bottleneck":
                c1, c2, c3 = blk.convs
                wgrad(c3, G3, h2, s2)
                G2 = _conv_dgrad(c3, G3, s2, gate=h2)
                wgrad(c2, G2, h1, s1)
                G1 = _conv_dgrad(c2, G2, s1, gate=h1)
            else:
                c1, c2 = blk.convs
                wgrad(c2, G3, h1, s1)
                G1 = _conv_dgrad(c2, G3, s1, gate=h1)
            wgrad(c1, G1, inp, ishape)
            if blk.ds is not None:
                wgrad(blk.ds, G3, inp, ishape)
            if need_dx:
                if blk.ds is not None and DS_DGRAD_INPLACE:
                    # conv1's gated data gradient, then the stride-2 downsample's added in place
                    # at the pixels its taps reach: gate(a + b) = gate(a) + b there, and the
                    # other three phases are final (no fill pass; bitwise the same values)
                    g = _conv_dgrad(c1, G1, ishape, gate=inp)
                    g = _conv_dgrad(blk.ds, G3, ishape, addend=g, gate=inp, out=g)
                elif blk.ds is not None:
                    tmp = _conv_dgrad(c1, G1, ishape)
                    g = _conv_dgrad(blk.ds, G3, ishape, addend=tmp, gate=inp)
                else:
                    g = _conv_dgrad(c1, G1, ishape, addend=G3, gate=inp)
            else:
                g = None
        if pending:
            _conv_wgrad_group(pending, grads)
            del pending
        ov.join()
        del keep
        out = [None, None]
        for w in runner.weights:
            gw = grads.get(w)
            out.append(gw if (gw is not None and w.requires_grad) else None)
        ctx.saved_acts = None
        return tuple(out)


class BackboneRunner:
    """Holds the conv plan of a backbone body; call ``run(images)`` -> NHWC features."""

    def __init__(self, body, cdtype):
        self.stem, self.blocks = build_plan(body)
        self.cdtype = cdtype
        ws = [self.stem.conv.weight]
        for b in self.blocks:
            ws.extend(b.params())
        self.weights = ws
        self.specs = [self.stem] + [c for b in self.blocks
                                    for c in b.convs + ([b.ds] if b.ds is not None else [])]
        self._s2d_w = None
        self.use_s2d = os.environ.get("RETR_S2D_STEM", "1") != "0"
        # fused stem conv + max-pool on the space-to-depth path (A/B switch)
        self.stem_pool = os.environ.get("RETR_STEM_POOL", "1") != "0"
        self._cat_w = {}
        self.cat_used = []          # blocks that took the fused tail in the last forward
        self.use_cat = os.environ.get("RETR_CAT_TAIL", "1") != "0"
        self.fused_used = []        # blocks run by retr_bottleneck_s1_fwd in the last forward
        self.use_fused = os.environ.get("RETR_FUSED_BOTTLENECK", "1") != "0"

    def fused_block(self, blk, ishape):
        """bf16 stride-1 bottleneck of width 64 -> 256 (ResNet-50/101 layer1) on a map with
        H % 8 == 0 and W % 16 == 0: one retr_bottleneck_s1_fwd launch.  The caller only asks
        for blocks whose activations backward does not need."""
        if not (self.use_fused and self.cdtype == torch.bfloat16 and blk.kind == "bottleneck"):
            return False
        c1, c2, c3 = blk.convs
        n, h, w, cin = ishape
        ok = (c1.k == 1 and c1.s == 1 and c1.cout == 64 and c1.cp == cin
              and c2.k == 3 and c2.s == 1 and c2.p == 1 and c2.d == 1 and c2.cin == 64
              and c2.cout == 64 and c3.k == 1 and c3.s == 1 and c3.cin == 64
              and c3.cout == 256 and h % 8 == 0 and w % 16 == 0)
        if not ok:
            return False
        if blk.ds is None:
            return cin == 256
        ds = blk.ds
        return (cin == 64 and ds.k == 1 and ds.s == 1 and ds.p == 0 and ds.cp == 64
                and ds.cout == 256)

    def cat_tail(self, blk, ishape, s2):
        """bf16 bottleneck with a 1x1 downsample (the first block of every layer): conv3 +
        downsample + residual add + ReLU as one 1x1 conv over [h2 | x sampled at the downsample
        stride] (retr_conv1x1_fwd_cat) -- the downsample output is never written or re-read.
        Backward never needs it (the block's backward reads x, h1, h2 and the output gradient)."""
        ds = blk.ds
        if not (self.use_cat and self.cdtype == torch.bfloat16 and blk.kind == "bottleneck"
                and ds is not None):
            return False
        c3 = blk.convs[2]
        return (ds.k == 1 and ds.p == 0 and ds.d == 1 and c3.k == 1 and c3.s == 1 and c3.p == 0
                and ds.out_hw(ishape[1], ishape[2]) == tuple(s2[1:3]) and ishape[3] == ds.cp
                and s2[3] == c3.cp)

    def s2d_stem(self, c, h, w):
        """bf16 torchvision stem (7x7, stride 2, pad 3, RGB) on even-sized images: run it as the
        space-to-depth conv (_stem_s2d)."""
        st = self.stem
        return (self.use_s2d and self.cdtype == torch.bfloat16 and st.k == 7 and st.s == 2
                and st.p == 3 and st.d == 1 and st.cin == 3 and c == 3 and h % 2 == 0
                and w % 2 == 0)

    def run(self, images):
        # activations are only kept when autograd will call backward
        self.save = torch.is_grad_enabled() and any(w.requires_grad for w in self.weights)
        return _Backbone.apply(images, self, *self.weights)
