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
