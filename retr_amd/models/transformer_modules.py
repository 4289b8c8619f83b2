"""Pre-norm residual sub-layers and decoder embeddings (models/transformer_modules.py).

These are parameter containers with the reference's attribute names (``sublayer``, ``norm``,
``dropout``; ``word_embeddings``, ``position_embeddings``, ``LayerNorm``) so ``state_dict`` keys
match.  Their arithmetic runs in the fused operators of ``retr_amd.ops`` (called from
``ConcatTransformer.run``), never through torch's MultiheadAttention / Linear forward.
"""
import torch
from torch import nn


def feed_forward(dim_input, dim_feedforward):
    """Linear -> ReLU -> Linear (models/transformer_modules.py:6-11)."""
    return nn.Sequential(nn.Linear(dim_input, dim_feedforward), nn.ReLU(),
                         nn.Linear(dim_feedforward, dim_input))


class AttResidualBase(nn.Module):
    def __init__(self, sublayer, dimension, dropout=0.1):
        super().__init__()
        self.sublayer = sublayer
        self.dropout = nn.Dropout(dropout)
        self.norm = nn.LayerNorm(dimension)


class SelfAttResidual(AttResidualBase):
    """x + Dropout(MHA(q=k=LN(x)+pos, v=LN(x)))  (:22-46) — see ops.self_attn_block."""


class CrossAttResidual(AttResidualBase):
    """q + Dropout(MHA(q=LN(q)+q_pos, k=kv+k_pos, v=kv))  (:49-74) — see ops.cross_attn_block."""


class FFResidual(nn.Module):
    """x + Dropout(FFN(LN(x)))  (:77-97) — see ops.ffn_block."""

    def __init__(self, sublayer, dimension, dropout=0.1):
        super().__init__()
        self.sublayer = sublayer
        self.dropout = nn.Dropout(dropout)
        self.norm = nn.LayerNorm(dimension)


class DecoderEmbeddings(nn.Module):
    """LN_eps(word[caps] + pos[0..T-1]) -> dropout  (:100-129) — see ops.embed_ln."""

    def __init__(self, config):
        super().__init__()
        self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_dim,
                                            padding_idx=config.pad_token_id)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, config.hidden_dim)
        self.LayerNorm = torch.nn.LayerNorm(config.hidden_dim, eps=config.layer_norm_eps)
        self.dropout = nn.Dropout(config.dropout)

    def forward(self, x):
        from .. import ops
        b, t = x.shape
        return ops.embed_ln(self, x, self.training).view(b, t, -1)
