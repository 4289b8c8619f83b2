"""Shared configs for parity tests (model configs of SURVEY.md §8 and micro variants)."""
import copy

from retr_amd.configuration import Config


def make_config(backbone="ResNet18", dilation=False, hidden=64, layers=(1, 1), vocab=1000,
                max_pos=16, nheads=8, ffn=128, dtype="fp32", dropout=0.0, lr_backbone=1e-5):
    c = Config()
    c.backbone = backbone
    c.dilation = dilation
    c.hidden_dim = hidden
    c.enc_layers, c.dec_layers = layers
    c.vocab_size = vocab
    c.max_position_embeddings = max_pos
    c.nheads = nheads
    c.dim_feedforward = ffn
    c.dtype = dtype
    c.dropout = dropout
    c.lr_backbone = lr_backbone
    return c


# name -> (config kwargs, image size, batch)
PARITY_CASES = {
    "micro_r18": (dict(backbone="ResNet18", hidden=64, layers=(1, 1), vocab=1000, max_pos=16,
                       ffn=128), 64, 2),
    "micro_r50_dil": (dict(backbone="ResNet50", dilation=True, hidden=64, layers=(2, 2),
                           vocab=1000, max_pos=16, ffn=128), 96, 2),
    "cfg1": (dict(backbone="ResNet18", hidden=128, layers=(1, 1), vocab=30522, max_pos=128,
                  ffn=2048), 224, 2),
}


def clone_config(c):
    return copy.deepcopy(c)


# Non-default reference surfaces: name -> (config kwargs, image size, batch, extra attributes)
VARIANT_CASES = {
    "micro_loc": (dict(backbone="ResNet18", hidden=64, layers=(1, 1), vocab=1000, max_pos=16,
                       ffn=128), 64, 2, {"use_location_features": True}),
    "micro_globalloc": (dict(backbone="ResNet18", hidden=64, layers=(1, 1), vocab=1000,
                             max_pos=16, ffn=128), 64, 2,
                        {"use_location_features": True, "use_global_features": True}),
    "micro_learned_pe": (dict(backbone="ResNet18", hidden=64, layers=(2, 1), vocab=1000,
                              max_pos=16, ffn=128), 64, 2, {"position_embedding": "learned"}),
    "micro_postnorm": (dict(backbone="ResNet18", hidden=64, layers=(2, 2), vocab=1000,
                            max_pos=16, ffn=128), 64, 2, {"pre_norm": False}),
}

# transformer half at real depth (models/ConcatTransformer.py import)
F2_CASE = dict(backbone="ResNet50", hidden=256, layers=(6, 6), vocab=30522, max_pos=128,
               ffn=2048)


def f2_inputs(cfg, B=2, S=196):
    """Deterministic inputs of the F2 slice: src [B, C, S] ~ N(0,1), key-padding mask with the
    last 20 tokens of sample 1 padded, captions, and the fixed weight of the backward probe."""
    import numpy as np
    import torch
    from retr_amd.synthetic import synthetic_captions
    r = np.random.default_rng([11, 1])
    src = torch.from_numpy(r.standard_normal((B, cfg.hidden_dim, S), dtype=np.float32))
    mask = torch.zeros(B, S, dtype=torch.bool)
    mask[1, S - 20:] = True
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=12)
    weight = torch.from_numpy(r.standard_normal((cfg.max_position_embeddings, B,
                                                 cfg.hidden_dim), dtype=np.float32))
    return src, mask, caps[:, :-1], cap_mask[:, :-1], weight


def variant_inputs(name, cfg):
    """Deterministic inputs of a VARIANT_CASES entry: (images, mask, extra, caps, cap_mask)
    where ``extra`` is the list of the variant's additional forward inputs in call order
    ((g_images, g_mask) for the global context, then loc_feats)."""
    import numpy as np
    import torch
    from retr_amd.synthetic import synthetic_captions, synthetic_images
    _, size, B, _ = VARIANT_CASES[name]
    images, mask = synthetic_images(B, size, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=2)
    extra = []
    if cfg.use_global_features:
        extra.append(synthetic_images(B, size, seed=3, pad_band=False))
    if cfg.use_location_features:
        nf = 7 if not cfg.use_global_features else 5
        extra.append(torch.from_numpy(np.random.default_rng([5, 3]).uniform(0, 1, (B, nf))
                                      .astype(np.float32)))
    return images, mask, extra, caps, cap_mask


def variant_config(name, dtype="fp32"):
    kw, _, _, extra = VARIANT_CASES[name]
    cfg = make_config(dtype=dtype, **kw)
    for k, v in extra.items():
        setattr(cfg, k, v)
    return cfg
