"""Position encodings (models/position_encoding.py).

``PositionalEncoding`` keeps the reference's fp32 sine table buffer ``pe`` [max_len, 1, C]
(:13-22, ``max_len=1024`` from ``build_position_encoding`` :69-70) so checkpoints load
unchanged.  On the hot path the table is consumed directly by the fused LayerNorm+pos-add
kernel (row s of the table for token s), so ``forward`` is only the API-compatible view.
"""
import math

import torch
from torch import nn


class PositionalEncoding(nn.Module):
    def __init__(self, d_model: int, max_len: int = 5000):
        super().__init__()
        position = torch.arange(max_len).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
        pe = torch.zeros(max_len, 1, d_model)
        pe[:, 0, 0::2] = torch.sin(position * div_term)
        pe[:, 0, 1::2] = torch.cos(position * div_term)
        self.register_buffer("pe", pe)

    def table(self, seq_len):
        """[S, C] rows used by the fused kernels; raises like the reference for S > max_len."""
        if seq_len > self.pe.shape[0]:
            raise RuntimeError(
                f"The size of tensor a ({seq_len}) must match the size of tensor b "
                f"({self.pe.shape[0]}) at non-singleton dimension 2")
        return self.pe[:seq_len, 0]

    def forward(self, x):
        """x: [B, C, S] -> encoding [B, C, S] (models/position_encoding.py:24-35)."""
        b, _, s = x.shape
        return self.table(s).t().unsqueeze(0).repeat(b, 1, 1)


class PositionalEmbedding(nn.Module):
    """Learned variant ('learned'/'v3', models/position_encoding.py:38-63): LayerNorm of the
    first S rows of ``pos_embed``, repeated over the batch, dropout (fixed p=0.1 like the
    reference).  On the hot path ConcatTransformer.position_rows runs it as ops.learned_pos
    (HIP LayerNorm + dropout kernels) and feeds the fused LayerNorm+pos kernels."""

    def __init__(self, embedding_dim, dropout=0.1, max_position_embeddings=5000):
        super().__init__()
        self.pos_embed = nn.Embedding(max_position_embeddings, embedding_dim)
        self.LayerNorm = nn.LayerNorm(embedding_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        """x: [B, C, S] -> embeddings [B, C, S] (reference layout)."""
        from .. import ops
        b, _, s = x.shape
        rows = ops.learned_pos(self, b, s, self.training)
        return rows.view(b, s, -1).permute(0, 2, 1)


def build_position_encoding(config):
    if config.position_embedding in ("v2", "sine"):
        print("Using sine/cosine positional encodings")
        return PositionalEncoding(config.hidden_dim, max_len=1024)
    if config.position_embedding in ("v3", "learned"):
        print("Using learned positional encodings")
        return PositionalEmbedding(config.hidden_dim, max_position_embeddings=1024, dropout=0.1)
    raise ValueError(f"not supported {config.position_embedding}")
