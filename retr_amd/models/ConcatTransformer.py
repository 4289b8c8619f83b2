"""Pre-norm DETR-style encoder-decoder (models/ConcatTransformer.py).

Same module tree / parameter names / init as the reference (``encoder.layers.i.self_attn``,
``encoder.layers.i.ff``, ``encoder.norm``, ``positional_encoding.pe``, ``embeddings``,
``decoder.layers.i.{tgt_self_attn, tgt_src_cross_attn, ff}``, ``decoder.norm``; xavier on every
parameter with dim > 1, :40-43).  ``run`` executes the hot path on the MI355X kernels in a
batch-major token layout ([B*L, C] rows, no seq-first permutes); ``forward`` keeps the
reference signature and output layout.
"""
from collections import defaultdict

import torch
from torch import nn

from .position_encoding import build_position_encoding
from .utils import _get_clones
from .transformer_modules import (feed_forward, SelfAttResidual, CrossAttResidual, FFResidual,
                                  DecoderEmbeddings)


class TransformerEncoderLayer(nn.Module):
    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu",
                 normalize_before=False):
        super().__init__()
        self.self_attn = SelfAttResidual(nn.MultiheadAttention(d_model, nhead, dropout=dropout),
                                         dimension=d_model, dropout=dropout)
        self.ff = FFResidual(feed_forward(dim_input=d_model, dim_feedforward=dim_feedforward),
                             dimension=d_model, dropout=dropout)


class TransformerDecoderLayer(nn.Module):
    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu",
                 normalize_before=False):
        super().__init__()
        self.tgt_self_attn = SelfAttResidual(
            nn.MultiheadAttention(d_model, nhead, dropout=dropout), dimension=d_model,
            dropout=dropout)
        self.tgt_src_cross_attn = CrossAttResidual(
            nn.MultiheadAttention(d_model, nhead, dropout=dropout), dimension=d_model,
            dropout=dropout)
        self.ff = FFResidual(feed_forward(dim_input=d_model, dim_feedforward=dim_feedforward),
                             dimension=d_model, dropout=dropout)


class TransformerEncoder(nn.Module):
    def __init__(self, encoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = _get_clones(encoder_layer, num_layers)
        self.num_layers = num_layers
        self.norm = norm


class TransformerDecoder(nn.Module):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = _get_clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.norm = norm


class ConcatTransformer(nn.Module):

    def __init__(self, config, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=2048, dropout=0.1, activation="relu", normalize_before=False):
        super().__init__()
        encoder_layer = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout,
                                                activation, normalize_before)
        encoder_norm = nn.LayerNorm(d_model) if normalize_before else None
        self.encoder = TransformerEncoder(encoder_layer, num_encoder_layers, encoder_norm)
        self.positional_encoding = build_position_encoding(config)
        self.embeddings = DecoderEmbeddings(config)
        decoder_layer = TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout,
                                                activation, normalize_before)
        self.decoder = TransformerDecoder(decoder_layer, num_decoder_layers, nn.LayerNorm(d_model))
        self._reset_parameters()
        self.d_model = d_model
        self.nhead = nhead

    def _reset_parameters(self):
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)

    # ------------------------------------------------------------------------------------------
    def position_rows(self, B, S):
        """(table, period): the encoder position encoding as rows consumed by the fused
        LayerNorm(+pos) kernels — row r of the token matrix uses table[r % period].  Sine
        (models/position_encoding.py:24-35): the fixed [S, C] slice, period S.  Learned
        ('learned'/'v3', :50-63): LayerNorm(pos_embed) repeated and dropped out per sample,
        [B*S, C], period B*S."""
        from .. import ops
        from .position_encoding import PositionalEmbedding
        pe_mod = self.positional_encoding
        if isinstance(pe_mod, PositionalEmbedding):
            return ops.learned_pos(pe_mod, B, S, self.training), B * S
        return pe_mod.table(S), S

    def encode(self, src_rows, B, S, kpm_src, cdtype, want_att=False):
        """Encoder stack + final norm.  src_rows: fp32 [B*S, C].  Returns (mem, mem_pos) in the
        compute dtype plus the list of head-averaged self-attention maps if ``want_att``."""
        from .. import ops
        pe, period = self.position_rows(B, S)
        x = src_rows
        atts = []
        layers = list(self.encoder.layers)
        for i, layer in enumerate(layers):
            sa = layer.self_attn
            r = ops.self_attn_block(sa, x, pe, period, B, S, kpm_src, False, self.training,
                                    cdtype, want_probs=want_att)
            if want_att:
                x, a = r
                atts.append(a)
            else:
                x = r
            ff = layer.ff
            # the LayerNorm that reads this FFN's output, for its down-projection's epilogue
            if i + 1 < len(layers):
                nxt = (layers[i + 1].self_attn.norm, pe, period, True, True)
            else:
                nxt = (self.encoder.norm, pe, period, True, True) if self.encoder.norm else None
            x = ops.ffn_block(ff, x, self.training, cdtype, nxt)
        if self.encoder.norm is None:
            # pre_norm=False: the reference builds no encoder norm (:23-24) and the decoder
            # reads the raw residual stream as memory
            mem, mem_pos = ops.add_pos(x, pe, period, cdtype)
        else:
            mem, mem_pos = ops.ln_pos(x, self.encoder.norm, cdtype, pos=pe, period=period)
        return mem, mem_pos, atts

    def decode(self, mem, mem_pos, B, S, kpm_src, tgt, tgt_mask, cdtype, want_att=False):
        """Decoder stack + final norm over the full T=max_position_embeddings sequence."""
        from .. import ops
        T = tgt.shape[1]
        qpos = self.embeddings.position_embeddings.weight
        if T != qpos.shape[0]:
            raise RuntimeError(f"The size of tensor a ({T}) must match the size of tensor b "
                               f"({qpos.shape[0]}) at non-singleton dimension 0")
        kpm_tgt = tgt_mask.contiguous().view(torch.uint8)
        y = ops.embed_ln(self.embeddings, tgt, self.training, shared=True)
        att_s, att_x = [], []
        layers = list(self.decoder.layers)
        for i, layer in enumerate(layers):
            sa = layer.tgt_self_attn
            r = ops.self_attn_block(sa, y, qpos, T, B, T, kpm_tgt, True, self.training, cdtype,
                                    want_probs=want_att)
            if want_att:
                y, a = r
                att_s.append(a)
            else:
                y = r
            ca = layer.tgt_src_cross_attn
            r = ops.cross_attn_block(ca, y, qpos, T, mem_pos, mem, B, T, S, kpm_src,
                                     self.training, cdtype, want_probs=want_att)
            if want_att:
                y, a = r
                att_x.append(a)
            else:
                y = r
            ff = layer.ff
            nxt = ((layers[i + 1].tgt_self_attn.norm, qpos, T, True, True) if i + 1 < len(layers)
                   else (self.decoder.norm, None, None, True, False))
            y = ops.ffn_block(ff, y, self.training, cdtype, nxt)
        hs = ops.ln_pos(y, self.decoder.norm, cdtype)
        return hs, att_s, att_x

    def run(self, src_rows, B, S, src_mask, tgt, tgt_mask, cdtype, return_attention=False):
        """Hot path.  Returns (hs [B*T, C] compute dtype, att dict or {})."""
        from .. import ops
        ops.begin_pass()
        src_rows = ops.wgrad_fence(src_rows)
        kpm_src = src_mask.reshape(B, S).contiguous().view(torch.uint8)
        mem, mem_pos, att_e = self.encode(src_rows, B, S, kpm_src, cdtype, return_attention)
        hs, att_s, att_x = self.decode(mem, mem_pos, B, S, kpm_src, tgt, tgt_mask, cdtype,
                                       return_attention)
        atts = {}
        if return_attention:
            atts = {"enc_tc_self_att": torch.stack(att_e),
                    "dec_exp_self_att": torch.stack(att_s),
                    "dec_exp_tc_cross_att": torch.stack(att_x)}
        return hs, atts

    def forward(self, src_t, mask_t, src_c, mask_c, tgt, tgt_mask):
        """Reference signature (:45-74): src [B, C, S] -> (out [T, B, C], att dict)."""
        from ..configuration import compute_dtype
        if src_c is not None:
            src = torch.cat([src_t, src_c], 2)
            mask = torch.cat([mask_t, mask_c], 1)
        else:
            src, mask = src_t, mask_t
        b, c, s = src.shape
        rows = src.permute(0, 2, 1).reshape(b * s, c).float().contiguous()
        cdtype = getattr(self, "cdtype", torch.bfloat16)
        hs, atts = self.run(rows, b, s, mask, tgt, tgt_mask, cdtype, return_attention=True)
        return hs.view(b, tgt.shape[1], c).permute(1, 0, 2), atts


def build_transformer(config):
    return ConcatTransformer(config, d_model=config.hidden_dim, dropout=config.dropout,
                             nhead=config.nheads, dim_feedforward=config.dim_feedforward,
                             num_encoder_layers=config.enc_layers,
                             num_decoder_layers=config.dec_layers,
                             normalize_before=config.pre_norm)
