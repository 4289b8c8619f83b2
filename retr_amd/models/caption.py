"""Caption model + MLP head + criterion (models/caption.py).

``build_model(config) -> (model, criterion)`` and ``Caption.forward(samples, target_exp,
target_exp_mask, return_attention=False)`` keep the reference contract:
logits [B, T, V] (compute dtype; the vocabulary rows are padded to a multiple of 64 in memory,
so the returned tensor is a [B, T, V] view), or ``(logits, att_dict)``.

Data flow (all on the MI355X kernels): images NCHW -> NHWC ResNet body (retr_amd.resnet) ->
input_proj as a GEMM over pixels ([B*S, Cb] x [Cb, C], its data-gradient gated by the
backbone's final ReLU) -> ConcatTransformer.run in batch-major rows -> fused MLP head.
"""
import torch
from torch import nn

from .utils import NestedTensor, nested_tensor_from_tensor_list
from .backbone import build_backbone
from .ConcatTransformer import build_transformer as build_concat_transformer
from ..configuration import compute_dtype


class MLP(nn.Module):
    """Very simple multi-layer perceptron (models/caption.py:161-174)."""

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(n, k) for n, k in zip([input_dim] + h,
                                                                     h + [output_dim]))
        # ops.mlp_head runs the last layer over output rows padded to a multiple of 64: with
        # FusedAdamW the parameter slots reserve those rows (always zero), so the padded bf16
        # weight and fp32 bias are views of the optimizer's arenas (no per-step copies)
        last = self.layers[-1]
        last.weight._retr_pad_rows = last.bias._retr_pad_rows = (output_dim + 63) // 64 * 64


class Caption(nn.Module):

    def __init__(self, backbone, transformer, positional_encoding, hidden_dim, vocab_size):
        super().__init__()
        self.backbone = backbone
        self.positional_encoding = positional_encoding
        self.input_proj = nn.Conv2d(in_channels=backbone.num_channels, out_channels=hidden_dim,
                                    kernel_size=1)
        self.transformer = transformer
        self.mlp = MLP(hidden_dim, 512, vocab_size, 3)
        self.cdtype = torch.bfloat16

    def set_compute_dtype(self, dtype):
        self.cdtype = dtype
        self.transformer.cdtype = dtype
        self.backbone.cdtype = dtype
        return self

    def encode_image(self, samples):
        """Backbone + input_proj -> (src rows fp32 [B*S, C], mask [B, S] bool, B, S)."""
        from .. import ops
        if not isinstance(samples, NestedTensor):
            samples = nested_tensor_from_tensor_list(samples)
        feats, mask = self.backbone.features(samples, self.cdtype)
        b, h, w, cb = feats.shape
        s = h * w
        src = ops.linear(feats.view(b * s, cb), self.input_proj.weight, self.input_proj.bias,
                         self.cdtype, out_f32=True, dgate=feats.view(b * s, cb))
        return src, mask.view(b, s), b, s

    def memory_tokens(self, samples):
        """Encoder input rows of this model: (src fp32 [B*S, C], mask [B, S], B, S)."""
        return self.encode_image(samples)

    def forward(self, samples, target_exp, target_exp_mask, return_attention=False):
        from .. import ops
        src, mask, b, s = self.encode_image(samples)
        assert mask is not None
        hs, att = self.transformer.run(src, b, s, mask, target_exp, target_exp_mask, self.cdtype,
                                       return_attention=return_attention)
        out = ops.mlp_head(self.mlp, hs, b, target_exp.shape[1], self.cdtype)
        if return_attention:
            return out, att
        return out


def _small_linear(x, lin, cdtype):
    """nn.Linear with a tiny input width (loc_proj: 7 or 1 features) on the MFMA GEMM: the
    feature dim is zero-padded to the GEMM's 16-byte K granule (the pad contributes exact
    zeros); the weight gradient flows back through the pad.  x: [M, K] -> fp32 [M, C]."""
    import torch.nn.functional as F
    from .. import ops
    k = lin.in_features
    if x.shape[-1] != k:       # F.linear's error (the reference's Linear(7) vs 5 features)
        raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied "
                           f"({x.shape[0]}x{x.shape[-1]} and {k}x{lin.out_features})")
    kp = (k + 7) // 8 * 8
    xp = F.pad(x.float(), (0, kp - k)).to(cdtype).contiguous()
    wp = F.pad(lin.weight, (0, kp - k))
    return ops.linear(xp, wp, lin.bias, cdtype, out_f32=True)


class _ConcatMixin:
    """Shared host plumbing of the location / global-context variants: build the memory token
    rows of ConcatTransformer.forward's concatenation (models/ConcatTransformer.py:47-53) in
    the batch-major layout of ConcatTransformer.run."""

    @staticmethod
    def _concat(parts):
        b = parts[0][0].shape[0]
        rows = torch.cat([r for r, _ in parts], 1)            # [B, S_total, C]
        mask = torch.cat([m for _, m in parts], 1)            # [B, S_total]
        s = rows.shape[1]
        return rows.reshape(b * s, -1), mask, b, s

    def _run(self, parts, target_exp, target_exp_mask, return_attention):
        from .. import ops
        rows, mask, b, s = self._concat(parts)
        hs, att = self.transformer.run(rows, b, s, mask, target_exp,
                                       target_exp_mask, self.cdtype,
                                       return_attention=return_attention)
        out = ops.mlp_head(self.mlp, hs, b, target_exp.shape[1], self.cdtype)
        if return_attention:
            return out, att
        return out

    def _image_part(self, samples):
        src, mask, b, s = self.encode_image(samples)
        return src.view(b, s, -1), mask

    def set_compute_dtype(self, dtype):
        self.cdtype = dtype
        self.transformer.cdtype = dtype
        self.backbone.cdtype = dtype
        return self


class CaptionLoc(_ConcatMixin, Caption):
    """Target image + location features (models/caption.py:50-95): ``loc_proj = Linear(7, C)``
    maps the location vector to one extra, never-masked memory token appended after the image
    tokens.  The dataset's position features have 5 entries (data_utils/utils.py:200-237), so
    with the reference's Linear(7) a real batch fails exactly as in the reference (F.linear's
    shape error); 7-feature inputs run."""

    def __init__(self, backbone, transformer, positional_encoding, hidden_dim, vocab_size):
        nn.Module.__init__(self)          # registration order = reference (parameter order)
        self.backbone = backbone
        self.positional_encoding = positional_encoding
        self.input_proj = nn.Conv2d(backbone.num_channels, hidden_dim, kernel_size=1)
        self.loc_proj = nn.Linear(7, hidden_dim)
        self.transformer = transformer
        self.mlp = MLP(hidden_dim, 512, vocab_size, 3)
        self.cdtype = torch.bfloat16

    def _parts(self, t_samples, loc_feats):
        t_rows, t_mask = self._image_part(t_samples)
        b = t_rows.shape[0]
        loc = _small_linear(loc_feats.reshape(b, -1), self.loc_proj, self.cdtype)   # [B, C]
        loc_mask = torch.zeros((b, 1), dtype=torch.bool, device=t_mask.device)
        return [(t_rows, t_mask), (loc.view(b, 1, -1), loc_mask)]

    def memory_tokens(self, t_samples, loc_feats):
        return self._concat(self._parts(t_samples, loc_feats))

    def forward(self, t_samples, loc_feats, target_exp, target_exp_mask, return_attention=False):
        return self._run(self._parts(t_samples, loc_feats), target_exp, target_exp_mask,
                         return_attention)


class CaptionGlobalLoc(_ConcatMixin, Caption):
    """Target image + location features + global context image (models/caption.py:98-158):
    memory = [target tokens, one token per location feature (``loc_proj = Linear(1, C)`` on
    each scalar), context-image tokens (second backbone pass, its mask passed through
    ensure_unmasked_values)]."""

    def __init__(self, backbone, transformer, positional_encoding, hidden_dim, vocab_size):
        nn.Module.__init__(self)          # registration order = reference (parameter order)
        self.backbone = backbone
        self.positional_encoding = positional_encoding
        self.input_proj = nn.Conv2d(backbone.num_channels, hidden_dim, kernel_size=1)
        self.loc_proj = nn.Linear(1, hidden_dim)
        self.transformer = transformer
        self.mlp = MLP(hidden_dim, 512, vocab_size, 3)
        self.cdtype = torch.bfloat16

    def forward(self, t_samples, g_samples, loc_feats, target_exp, target_exp_mask,
                return_attention=False):
        return self._run(self._parts(t_samples, g_samples, loc_feats), target_exp,
                         target_exp_mask, return_attention)

    def memory_tokens(self, t_samples, g_samples, loc_feats):
        return self._concat(self._parts(t_samples, g_samples, loc_feats))

    def _parts(self, t_samples, g_samples, loc_feats):
        from .utils import ensure_unmasked_values
        t_rows, t_mask = self._image_part(t_samples)
        b = t_rows.shape[0]
        nf = loc_feats.shape[1]
        loc = _small_linear(loc_feats.reshape(b * nf, 1), self.loc_proj, self.cdtype)
        loc_mask = torch.zeros((b, nf), dtype=torch.bool, device=t_mask.device)
        if not isinstance(g_samples, NestedTensor):
            g_samples = nested_tensor_from_tensor_list(g_samples)
        feats, g_mask = self.backbone.features(g_samples, self.cdtype)
        gb, gh, gw, cb = feats.shape
        g_mask = ensure_unmasked_values(g_mask)
        from .. import ops
        g_rows = ops.linear(feats.view(gb * gh * gw, cb), self.input_proj.weight,
                            self.input_proj.bias, self.cdtype, out_f32=True,
                            dgate=feats.view(gb * gh * gw, cb))
        return [(t_rows, t_mask), (loc.view(b, nf, -1), loc_mask),
                (g_rows.view(gb, gh * gw, -1), g_mask.view(gb, gh * gw))]


class CrossEntropyLoss(nn.CrossEntropyLoss):
    """``torch.nn.CrossEntropyLoss()`` semantics (mean, no ignore_index hit for pad id 0) on the
    fused HIP kernel; called exactly as engine.py:71 does: criterion(out.permute(0,2,1), tgt)."""

    def forward(self, input, target):
        from .. import ops
        if input.dim() != 3 or self.reduction != "mean" or self.weight is not None \
                or self.label_smoothing != 0.0:
            raise NotImplementedError("only the reference's CrossEntropyLoss() call is supported")
        return ops.cross_entropy(input, target)


def build_model(config):
    backbone = build_backbone(config)
    transformer = build_concat_transformer(config)
    use_global = config.use_global_features
    use_location = config.use_location_features
    print(f"global features: {use_global}, location features: {use_location}")
    if not use_global and not use_location:
        Model = Caption
    elif not use_global and use_location:
        Model = CaptionLoc
    elif use_global and use_location:
        Model = CaptionGlobalLoc
    else:
        raise NotImplementedError()
    model = Model(backbone, transformer, None, config.hidden_dim, config.vocab_size)
    model.set_compute_dtype(compute_dtype(config))
    if getattr(config, "deterministic", False):
        from .. import ops
        ops.set_deterministic(True)
    print(f"Built {model.__class__.__name__} model with {transformer.__class__.__name__}")
    criterion = CrossEntropyLoss()
    return model, criterion
