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


class CaptionLoc(nn.Module):
    """Parameter container of the location-feature variant (models/caption.py:50-95); its
    forward is out of the hot-path scope."""

    def __init__(self, backbone, transformer, positional_encoding, hidden_dim, vocab_size):
        super().__init__()
        self.backbone = backbone
        self.positional_encoding = positional_encoding
        self.input_proj = nn.Conv2d(backbone.num_channels, hidden_dim, kernel_size=1)
        self.loc_proj = nn.Linear(7, hidden_dim)
        self.transformer = transformer
        self.mlp = MLP(hidden_dim, 512, vocab_size, 3)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("CaptionLoc is not on the MI355X hot path (SURVEY.md §8 f3)")


class CaptionGlobalLoc(CaptionLoc):
    """Parameter container of models/caption.py:98-158 (``loc_proj = Linear(1, C)``)."""

    def __init__(self, backbone, transformer, positional_encoding, hidden_dim, vocab_size):
        super().__init__(backbone, transformer, positional_encoding, hidden_dim, vocab_size)
        self.loc_proj = nn.Linear(1, hidden_dim)


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
    if isinstance(model, Caption):
        model.set_compute_dtype(compute_dtype(config))
    print(f"Built {model.__class__.__name__} model with {transformer.__class__.__name__}")
    criterion = CrossEntropyLoss()
    return model, criterion
