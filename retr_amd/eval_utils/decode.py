"""Greedy decoding (eval_utils/decode.py) on the MI355X kernels.

``greedy`` keeps the reference signature and output contract (decode.py:53-81): caption
[B, max_len] int64, column 0 = BOS; at step i, if every row has produced EOS (at this or an
earlier step) the loop returns without writing column i+1, otherwise the step's argmax is
written to column i+1 for all rows.

Instead of the reference's 127 full model forwards (backbone included) it runs the
mathematically identical incremental form (the decoder is causal, masked
positions have exactly zero influence, rows are independent):
  * backbone + input_proj + encoder + cross-attention K/V once per batch;
  * per step one query row per caption through the decoder with a self-attention K/V cache,
    the final LayerNorm, the MLP head and a first-index argmax;
  * the finished/early-exit bookkeeping runs on the device (retr_greedy_update) and the host
    polls it every ``poll`` steps, so no per-step synchronisation.
The T-1 per-step launch sequences are captured once per (shape, weights) as hipGraphs and
replayed, so a step costs its kernels' device time, not ~100 host launches.  The single-query
attention (retr_attention_decode) reduces keys in a different order than the tiled training
kernel, so logits agree with the full recompute to rounding, and the token ids agree with the
reference algorithm run by the CPU oracle (tests/test_gpu_model.py).
"""
import torch

from .. import ops
from .._lib import call, load, ptr
from ..ops import dcode, k_linear_fwd, _st


def create_caption_and_mask(start_token, max_length, batch_size=1):
    caption = torch.zeros((batch_size, max_length), dtype=torch.long)
    mask = torch.ones((batch_size, max_length), dtype=torch.bool)
    caption[:, 0] = start_token
    mask[:, 0] = False
    return caption, mask


def prepare_tokenizer():
    """Reference helper (decode.py:6-10); needs the HF hub (network) — out of hot-path scope."""
    from transformers import BertTokenizer
    tokenizer = BertTokenizer.from_pretrained("bert-base-uncased")
    start_token = tokenizer.convert_tokens_to_ids(tokenizer._cls_token)
    end_token = tokenizer.convert_tokens_to_ids(tokenizer._sep_token)
    return tokenizer, start_token, end_token


# The fused step's attention sub-layers as one wave per (row, head) (csrc/decode_heads.hip);
# False: the round-4 block-per-row kernels (csrc/decode.hip dec_gemm + dec_attn_row)
DEC_HEADS = True
# (with DEC_HEADS) the cross-attention residual + LN3 in the FFN kernel's prologue
DEC_FFN_LN = True
# (with DEC_FFN_LN) the FFN residual + the next layer's LN1 in the self-attention prologue
DEC_FOLD_ROWS = True
# fp32 parity mode: the step's linears on the skinny exact-f32 kernel
DEC_F32_SKINNY = True
# decode steps per captured hipGraph (the host polls the early-exit flag between graphs):
# one replay launch per 8 steps instead of per step
DEC_GRAPH_STEPS = 8
# greedy batches decoded as DEC_SPLIT independent row groups on concurrent streams of one graph
# (each group at least DEC_SPLIT_MIN_ROWS rows); 1 = one group
DEC_SPLIT = 1   # 2 measured SLOWER (bf16 2290 -> 1486, fp32 1217 -> ~1000 refs/s: profiles/r6_ab_dec_split_rejected.txt)
DEC_SPLIT_MIN_ROWS = 16
# fp32 parity mode: three fused launches per decoder layer (csrc/decode_f32.hip, round 6)
# instead of the per-op step
DEC_F32_FUSED = True
# the greedy step's MLP-head layers 1-2 on the skinny bf16 linear
DEC_HEAD_SKINNY = True
# rows up to which the folded (three-launch) layer is used (beyond: five launches per layer)
DEC_FOLD_MAX_ROWS = 512
# rows beyond which the folded FFN runs 128 hidden units per block
DEC_FFN_HB128_ROWS = 64
# (with DEC_FOLD_ROWS) the decoder embeddings + first LN1 in the first self-attention launch
DEC_EMBED_FOLD = False   # measured neutral (0.248 ms/step either way): the token -> word-row load is a dependent round trip

# Rows per block of the attention sub-layer kernels: None = automatic (beam groups of K rows
# share the head's staged weights and memory keys / values: K in {2, 4, 5}), else an int for
# every launch (1 = a block per (row, head)).
DEC_ROWS_PER_BLOCK = None


def _rows_per_block(R, C, H, K, nkeys, S):
    """(self, cross) rows per block for retr_dec_self_heads_mr / retr_dec_cross_heads_mr."""
    if C != 256 or H != 8:
        return 1, 1
    rb = DEC_ROWS_PER_BLOCK
    if rb is None:
        rb = K if K in (2, 4, 5) else 1
    if rb == 1 or R % rb:
        return 1, 1
    return (rb if nkeys <= 128 else 1), (rb if S <= 256 else 1)


class _DecodeState:
    """Static device buffers (and captured per-step hipGraphs) for one (B, K, S, T) shape;
    the decoder runs R = B*K rows (K = beams per image, 1 for greedy)."""

    def __init__(self, B, S, T, C, F, n_layers, V, cd, dev, K=1):
        f32 = torch.float32
        R = B * K
        self.B, self.K, self.R, self.S, self.T = B, K, R, S, T
        self.kx = [torch.empty(B * S, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.vx = [torch.empty(B * S, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.kc = [torch.zeros(R * T, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.vc = [torch.zeros(R * T, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.kpm = torch.zeros(B, S, dtype=torch.uint8, device=dev)
        self.caption = torch.zeros(B, T, dtype=torch.long, device=dev)
        self.tok = torch.zeros(R, dtype=torch.long, device=dev)
        self.finished = torch.zeros(R, dtype=torch.uint8, device=dev)
        self.done = torch.full((1,), -1, dtype=torch.int32, device=dev)
        self.y = torch.empty(R, C, dtype=f32, device=dev)
        self.y2 = torch.empty_like(self.y)
        self.n = torch.empty(R, C, dtype=cd, device=dev)
        self.npos = torch.empty_like(self.n)
        self.q = torch.empty_like(self.n)
        self.o = torch.empty_like(self.n)
        self.mean = torch.empty(R, dtype=f32, device=dev)
        self.rstd = torch.empty_like(self.mean)
        self.ffh = torch.empty(R, F, dtype=cd, device=dev)
        self.q2 = torch.empty_like(self.n)
        self.slabs = torch.empty(F // 32, R, C, dtype=f32, device=dev)   # fused FFN partials
        self.hslab = None       # per-head out-projection partials (DEC_HEADS), made on first use
        self.hslab2 = None
        self.h1 = torch.empty(R, 512, dtype=cd, device=dev)
        self.h2 = torch.empty(R, 512, dtype=cd, device=dev)
        self.Vp = (V + 63) // 64 * 64
        self.logits = torch.empty(R, self.Vp, dtype=cd, device=dev)
        self.pred = torch.empty(R, dtype=torch.long, device=dev)
        self.am_ws = torch.empty(max(1, load().retr_argmax_workspace(R) // 4),
                                 dtype=torch.float32, device=dev)   # split argmax partials
        if K > 1:
            self.init_beam(dev)
        self.head_bias = None
        self.graphs = None
        self.signature = None
        self.write_all = False    # a row group of a split batch (IncrementalGreedy._call_split)

    def init_beam(self, dev):
        R, K, T = self.R, self.K, self.T
        self.beam = True
        self.hist = torch.zeros(R, T, dtype=torch.long, device=dev)
        self.anc = torch.zeros(R, T, dtype=torch.int32, device=dev)
        self.scores = torch.zeros(R, dtype=torch.float32, device=dev)
        self.cand_tok = torch.zeros(R, K, dtype=torch.int32, device=dev)
        self.cand_lp = torch.zeros(R, K, dtype=torch.float32, device=dev)
        self.item_done = torch.zeros(self.B, dtype=torch.uint8, device=dev)


class IncrementalGreedy:
    """KV-cache greedy decoder over a ``Caption`` model (eval mode semantics).  The T-1 decode
    steps are captured once per (shape, weights) as hipGraphs and replayed per batch."""

    beam = False
    K = 1

    def __init__(self, model, use_graphs=True, fused=True):
        self.model = model
        self.tr = model.transformer
        self.cdtype = model.cdtype
        self.use_graphs = use_graphs
        self.fused = fused
        if not hasattr(model, "_retr_decode_states"):
            model._retr_decode_states = {}
        self.states = model._retr_decode_states

    def _ln(self, x, norm, y=None, y2=None, pos=None):
        M, C = x.shape
        call("retr_layernorm_fwd", dcode(self.cdtype), ptr(x), C, ptr(norm.weight),
             ptr(norm.bias), float(norm.eps), M, C, ptr(y), C, ptr(y2), ptr(pos), 1, None, None,
             _st())

    def _signature(self):
        return tuple((p._version, p.data_ptr()) for p in self.model.parameters())

    def _fusable(self, st):
        layers = list(self.tr.decoder.layers)
        C = st.n.shape[1]
        H = layers[0].tgt_self_attn.sublayer.num_heads
        F = layers[0].ff.sublayer[0].weight.shape[0]
        return (self.fused and self.cdtype == torch.bfloat16 and C in (256, 512)
                and C // H in (32, 64) and H % 4 == 0 and F % 32 == 0 and st.S <= 512
                and st.T <= 512 and self.model.mlp.layers[0].weight.shape[0] % 32 == 0)

    def _fusable_f32(self, st):
        """The fused fp32 parity-mode step (csrc/decode_f32.hip): d_model 256 in 8 heads, FFN
        width a multiple of 64, at most 512 self / memory keys; other shapes take the per-op
        step."""
        layers = list(self.tr.decoder.layers)
        C = st.n.shape[1]
        H = layers[0].tgt_self_attn.sublayer.num_heads
        F = layers[0].ff.sublayer[0].weight.shape[0]
        return (self.fused and DEC_F32_FUSED and self.cdtype == torch.float32 and C == 256
                and H == 8 and F % 64 == 0 and st.S <= 512 and st.T <= 512)

    def _heads_ok(self, st):
        """The per-(row, head) kernels (csrc/decode_heads.hip) hold at most 4 key chunks per wave:
        512 self / memory keys at head dim 32, 256 at head dim 64 (retr_dec_self_heads_ln /
        retr_dec_cross_heads); longer memories or captions take the block-per-row step (up to
        512 keys, retr_dec_attn_row)."""
        layers = list(self.tr.decoder.layers)
        hd = st.n.shape[1] // layers[0].tgt_self_attn.sublayer.num_heads
        return hd == 32 or (st.S <= 256 and st.T <= 256)

    def _lin(self, x, w, bias, y, relu=0, res=None):
        """The unfused step's linears; the fp32 parity mode's (few rows) on the skinny exact-f32
        kernel (csrc/decode.hip dec_linear_f32), everything else on the generic GEMM."""
        M, K = x.shape
        if (DEC_F32_SKINNY and x.dtype == torch.float32 and y.dtype == torch.float32
                and M <= 64 and K % 16 == 0 and x.stride(1) == 1 and w.stride(1) == 1
                and x.stride(0) % 4 == 0 and w.stride(0) % 4 == 0):
            call("retr_dec_linear_f32", ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(bias),
                 ptr(y), y.stride(0), M, w.shape[0], K, int(relu), ptr(res),
                 res.stride(0) if res is not None else 0, _st())
            return
        k_linear_fwd(x, w, bias, y, relu=relu, res=res)

    def _lin3(self, items):
        """q | k | v projections (same rows and K) in one skinny fp32 launch when they qualify."""
        x0, w0 = items[0][0], items[0][1]
        M, K = x0.shape
        ok = (DEC_F32_SKINNY and M <= 64 and K % 16 == 0 and all(
            x.dtype == torch.float32 and y.dtype == torch.float32 and x.shape == (M, K)
            and w.shape[1] == K and x.stride(1) == 1 and w.stride(1) == 1
            and x.stride(0) % 4 == 0 and w.stride(0) % 4 == 0 for x, w, b, y in items))
        if not ok:
            for x, w, b, y in items:
                self._lin(x, w, b, y)
            return
        args = []
        for x, w, b, y in items:
            args += [ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(b), ptr(y), y.stride(0),
                     w.shape[0], 0, None, 0]
        args += [None, 0, None, 0, None, None, 0, 0, 0, None, 0] * (3 - len(items))
        call("retr_dec_linear3_f32", len(items), *args, M, K, _st())

    def _step(self, st, i, eos_token):
        """Kernels of decode step i (reads token i, writes caption column i+1)."""
        if self._fusable(st):
            return self._step_fused(st, i, eos_token)
        if self._fusable_f32(st):
            return self._step_f32(st, i, eos_token)
        model, tr, cd = self.model, self.tr, self.cdtype
        B, S, T, R = st.B, st.S, st.T, st.R
        C = st.n.shape[1]
        layers = list(tr.decoder.layers)
        H = layers[0].tgt_self_attn.sublayer.num_heads
        hd = C // H
        emb = tr.embeddings
        qp = emb.position_embeddings.weight.detach()[i]
        s = _st()
        y, y2 = st.y, st.y2
        call("retr_embed_ln_fwd", ptr(st.tok), R, 1, C, ptr(emb.word_embeddings.weight), ptr(qp),
             ptr(emb.LayerNorm.weight), ptr(emb.LayerNorm.bias), float(emb.LayerNorm.eps), 0.0, 0,
             ptr(y), ptr(st.mean), ptr(st.rstd), s)
        for li, layer in enumerate(layers):
            sa = layer.tgt_self_attn
            sub = sa.sublayer
            w = ops.WEIGHTS.get(sub.in_proj_weight, cd)
            b = sub.in_proj_bias.detach()
            self._ln(y, sa.norm, y=st.n, y2=st.npos, pos=qp)
            self._lin3([(st.npos, w[:C], b[:C], st.q),
                        (st.npos, w[C:2 * C], b[C:2 * C], st.kc[li][i::T]),
                        (st.n, w[2 * C:], b[2 * C:], st.vc[li][i::T])])
            call("retr_attention_decode", dcode(cd), ptr(st.q), C, ptr(st.kc[li]), C,
                 ptr(st.vc[li]), C, ptr(st.o), C, R, H, i + 1, T, hd, None, 1,
                 ptr(st.anc) if self.beam else None, s)
            self._lin(st.o, ops.WEIGHTS.get(sub.out_proj.weight, cd),
                         sub.out_proj.bias.detach(), y2, res=y)
            y, y2 = y2, y
            ca = layer.tgt_src_cross_attn
            sub = ca.sublayer
            w = ops.WEIGHTS.get(sub.in_proj_weight, cd)
            b = sub.in_proj_bias.detach()
            self._ln(y, ca.norm, y2=st.npos, pos=qp)
            self._lin(st.npos, w[:C], b[:C], st.q)
            call("retr_attention_decode", dcode(cd), ptr(st.q), C, ptr(st.kx[li]), C,
                 ptr(st.vx[li]), C, ptr(st.o), C, R, H, S, S, hd, ptr(st.kpm), st.K, None, s)
            self._lin(st.o, ops.WEIGHTS.get(sub.out_proj.weight, cd),
                         sub.out_proj.bias.detach(), y2, res=y)
            y, y2 = y2, y
            ff = layer.ff
            self._ln(y, ff.norm, y=st.n)
            f0, f2 = ff.sublayer[0], ff.sublayer[2]
            self._lin(st.n, ops.WEIGHTS.get(f0.weight, cd), f0.bias.detach(), st.ffh, relu=1)
            self._lin(st.ffh, ops.WEIGHTS.get(f2.weight, cd), f2.bias.detach(), y2, res=y)
            y, y2 = y2, y
        l1, l2, l3 = model.mlp.layers
        V = l3.weight.shape[0]
        self._ln(y, tr.decoder.norm, y=st.n)
        self._lin(st.n, ops.WEIGHTS.get(l1.weight, cd), l1.bias.detach(), st.h1, relu=1)
        self._lin(st.h1, ops.WEIGHTS.get(l2.weight, cd), l2.bias.detach(), st.h2, relu=1)
        self._lin(st.h2, ops.WEIGHTS.get(l3.weight, cd, rows=st.Vp),
                     st.head_bias, st.logits)
        self._select(st, i, V, eos_token, s)

    def _step_f32(self, st, i, eos_token):
        """Decode step i of the fp32 parity mode as three fused launches per decoder layer
        (csrc/decode_f32.hip): retr_dec_self_f32 (previous FFN partials + residual -- or, at
        layer 0, the token embedding -- + LN1, the head's q | k | v, cache append, attention,
        partial out-projection), retr_dec_cross_f32 (head-partial sum + residual + LN2, cross
        query, attention over the memory, partial out-projection), retr_dec_ffn_f32 (head-partial
        sum + residual + LN3, FFN partials over 64 hidden units per block); then the final
        residual + decoder LN (retr_dec_rows_f32), the MLP head on the skinny exact-f32 linear and
        the selection.  Every value fp32."""
        model, tr = self.model, self.tr
        S, T, R = st.S, st.T, st.R
        C = st.n.shape[1]
        layers = list(tr.decoder.layers)
        H = layers[0].tgt_self_attn.sublayer.num_heads
        F = layers[0].ff.sublayer[0].weight.shape[0]
        W = lambda p: ops.WEIGHTS.get(p, torch.float32)        # noqa: E731
        if st.hslab is None:
            st.hslab = torch.empty(H, R, C, dtype=torch.float32, device=st.n.device)
            st.hslab2 = torch.empty_like(st.hslab)
        emb = tr.embeddings
        qp = emb.position_embeddings.weight.detach()[i]
        s = _st()
        x, xa = st.y, st.y2
        anc = ptr(st.anc) if self.beam else None
        nslab = F // 64
        for li, layer in enumerate(layers):
            sa, ca, ff = layer.tgt_self_attn, layer.tgt_src_cross_attn, layer.ff
            sub, csub = sa.sublayer, ca.sublayer
            f0, f2 = ff.sublayer[0], ff.sublayer[2]
            if li == 0:
                pro = (None, None, 0, None, ptr(st.tok), ptr(emb.word_embeddings.weight),
                       ptr(emb.LayerNorm.weight), ptr(emb.LayerNorm.bias),
                       float(emb.LayerNorm.eps))
            else:
                pf2 = layers[li - 1].ff.sublayer[2]
                pro = (ptr(x), ptr(st.slabs), nslab, ptr(pf2.bias), None, None, None, None, 0.0)
            call("retr_dec_self_f32", R, C, H, ptr(W(sub.in_proj_weight)), ptr(sub.in_proj_bias),
                 ptr(st.kc[li]), ptr(st.vc[li]), i, T, anc, ptr(W(sub.out_proj.weight)),
                 ptr(st.hslab), *pro, ptr(sa.norm.weight), ptr(sa.norm.bias), float(sa.norm.eps),
                 ptr(qp), ptr(xa), s)
            x, xa = xa, x
            call("retr_dec_cross_f32", R, C, H, ptr(st.hslab), ptr(x), ptr(sub.out_proj.bias),
                 ptr(xa), ptr(ca.norm.weight), ptr(ca.norm.bias), float(ca.norm.eps), ptr(qp),
                 ptr(W(csub.in_proj_weight)), ptr(csub.in_proj_bias), ptr(st.kx[li]),
                 ptr(st.vx[li]), S, st.K, ptr(st.kpm), ptr(W(csub.out_proj.weight)),
                 ptr(st.hslab2), s)
            x, xa = xa, x
            call("retr_dec_ffn_f32", ptr(x), ptr(st.hslab2), H, ptr(csub.out_proj.bias),
                 ptr(ff.norm.weight), ptr(ff.norm.bias), float(ff.norm.eps), ptr(xa), R, C,
                 ptr(W(f0.weight)), ptr(f0.bias), ptr(W(f2.weight)), F, ptr(st.slabs), s)
            x, xa = xa, x
        nx, f2 = tr.decoder.norm, layers[-1].ff.sublayer[2]
        call("retr_dec_rows_f32", ptr(x), ptr(st.slabs), nslab, ptr(f2.bias), R, C, ptr(xa),
             ptr(nx.weight), ptr(nx.bias), float(nx.eps), ptr(st.n), s)
        l1, l2, l3 = model.mlp.layers
        V = l3.weight.shape[0]
        self._lin(st.n, W(l1.weight), l1.bias.detach(), st.h1, relu=1)
        self._lin(st.h1, W(l2.weight), l2.bias.detach(), st.h2, relu=1)
        self._lin(st.h2, ops.WEIGHTS.get(l3.weight, torch.float32, rows=st.Vp), st.head_bias,
                  st.logits)
        self._select(st, i, V, eos_token, s)

    def _step_fused(self, st, i, eos_token):
        """Decode step i as five fused launches per decoder layer (csrc/decode.hip):
        [q|k|v] GEMM (+cache append); self-attention + out-proj + residual + LN2 + cross query;
        cross-attention + out-proj + residual + LN3; FFN split over hidden units; ordered slab
        reduce + residual + the next LayerNorm.  With DEC_HEADS (default) the first three are
        one wave per (row, head) instead (csrc/decode_heads.hip): the head's q|k|v + cache
        append + self-attention + partial out-projection; the self-attention residual + LN2 +
        the head's cross query + cross-attention + partial out-projection; then the head
        partials' ordered sum + residual + LN3 by retr_dec_rows."""
        if DEC_HEADS and self._heads_ok(st):
            return self._step_heads(st, i, eos_token)
        model, tr, cd = self.model, self.tr, self.cdtype
        S, T, R = st.S, st.T, st.R
        C = st.n.shape[1]
        layers = list(tr.decoder.layers)
        H = layers[0].tgt_self_attn.sublayer.num_heads
        F = layers[0].ff.sublayer[0].weight.shape[0]
        W = lambda p: ops.WEIGHTS.get(p, cd)        # noqa: E731
        emb = tr.embeddings
        qp = emb.position_embeddings.weight.detach()[i]
        s = _st()
        x, xa = st.y, st.y2
        n0 = layers[0].tgt_self_attn.norm
        call("retr_dec_embed_rows", ptr(st.tok), R, C, ptr(emb.word_embeddings.weight), ptr(qp),
             ptr(emb.LayerNorm.weight), ptr(emb.LayerNorm.bias), float(emb.LayerNorm.eps), ptr(x),
             ptr(n0.weight), ptr(n0.bias), float(n0.eps), ptr(st.n), ptr(st.npos), s)
        anc = ptr(st.anc) if self.beam else None
        nslab = F // 32
        for li, layer in enumerate(layers):
            sa, ca, ff = layer.tgt_self_attn, layer.tgt_src_cross_attn, layer.ff
            sub, csub = sa.sublayer, ca.sublayer
            kc, vc = st.kc[li], st.vc[li]
            call("retr_dec_gemm", ptr(st.n), ptr(st.npos), R, C, ptr(W(sub.in_proj_weight)),
                 ptr(sub.in_proj_bias), 3 * C, ptr(st.q), C, 1, ptr(kc) + 2 * i * C, T * C, 1,
                 ptr(vc) + 2 * i * C, T * C, 0, C, 0, s)
            call("retr_dec_attn_row", ptr(st.q), ptr(kc), ptr(vc), R, C, H, i + 1, T, 1, anc,
                 None, ptr(x), ptr(W(sub.out_proj.weight)), ptr(sub.out_proj.bias), ptr(xa),
                 ptr(ca.norm.weight), ptr(ca.norm.bias), float(ca.norm.eps), ptr(qp),
                 ptr(W(csub.in_proj_weight)), ptr(csub.in_proj_bias), ptr(st.q2), s)
            x, xa = xa, x
            call("retr_dec_attn_row", ptr(st.q2), ptr(st.kx[li]), ptr(st.vx[li]), R, C, H, S, S,
                 st.K, None, ptr(st.kpm), ptr(x), ptr(W(csub.out_proj.weight)),
                 ptr(csub.out_proj.bias), ptr(xa), ptr(ff.norm.weight), ptr(ff.norm.bias),
                 float(ff.norm.eps), None, None, None, ptr(st.o), s)
            x, xa = xa, x
            f0, f2 = ff.sublayer[0], ff.sublayer[2]
            call("retr_dec_ffn", ptr(st.o), R, C, ptr(W(f0.weight)), ptr(f0.bias),
                 ptr(W(f2.weight)), F, ptr(st.slabs), s)
            # residual + FFN partials, then the next layer's LN1 (+pos) or the final LN
            if li + 1 < len(layers):
                nx, npos = layers[li + 1].tgt_self_attn.norm, ptr(st.npos)
            else:
                nx, npos = tr.decoder.norm, None
            call("retr_dec_rows", ptr(x), ptr(st.slabs), nslab, ptr(f2.bias), R, C, ptr(xa),
                 ptr(nx.weight), ptr(nx.bias), float(nx.eps), ptr(qp) if npos else None,
                 ptr(st.n), npos, s)
            x, xa = xa, x
        l1, l2, l3 = model.mlp.layers
        V = l3.weight.shape[0]
        H1 = l1.weight.shape[0]
        call("retr_dec_gemm", ptr(st.n), None, R, C, ptr(W(l1.weight)), ptr(l1.bias), H1,
             ptr(st.h1), H1, 0, None, 0, 0, None, 0, 0, H1, 1, s)
        k_linear_fwd(st.h1, W(l2.weight), l2.bias.detach(), st.h2, relu=1)
        k_linear_fwd(st.h2, ops.WEIGHTS.get(l3.weight, cd, rows=st.Vp), st.head_bias, st.logits)
        self._select(st, i, V, eos_token, s)

    def _step_heads(self, st, i, eos_token):
        model, tr, cd = self.model, self.tr, self.cdtype
        S, T, R = st.S, st.T, st.R
        C = st.n.shape[1]
        layers = list(tr.decoder.layers)
        H = layers[0].tgt_self_attn.sublayer.num_heads
        F = layers[0].ff.sublayer[0].weight.shape[0]
        W = lambda p: ops.WEIGHTS.get(p, cd)        # noqa: E731
        if st.hslab is None:
            st.hslab = torch.empty(H, R, C, dtype=torch.float32, device=st.n.device)
            st.hslab2 = torch.empty_like(st.hslab)
        emb = tr.embeddings
        qp = emb.position_embeddings.weight.detach()[i]
        s = _st()
        x, xa = st.y, st.y2
        n0 = layers[0].tgt_self_attn.norm
        anc = ptr(st.anc) if self.beam else None
        nslab = F // 32
        # three launches per layer (up to 64 rows): the FFN residual + next LN1 in the next
        # layer's self-attention prologue, the cross residual + LN3 in the FFN prologue
        fold = DEC_FFN_LN and DEC_FOLD_ROWS and R <= DEC_FOLD_MAX_ROWS and F % 64 == 0
        rbs, rbx = _rows_per_block(R, C, H, st.K, i + 1, S)
        # hidden units per folded-FFN block: 128 beyond DEC_FFN_HB128_ROWS rows (half the blocks
        # re-deriving each row group's LayerNorm, half the partial slabs), else 64
        hb = 128 if (R > DEC_FFN_HB128_ROWS and C == 256 and F % 128 == 0 and H <= 8) else 64
        # the embeddings + first LN1 in the first self-attention launch (per-row blocks)
        embed = fold and DEC_EMBED_FOLD and rbs == 1 and C // H == 32 and i < 128
        if not embed:
            call("retr_dec_embed_rows", ptr(st.tok), R, C, ptr(emb.word_embeddings.weight),
                 ptr(qp), ptr(emb.LayerNorm.weight), ptr(emb.LayerNorm.bias),
                 float(emb.LayerNorm.eps), ptr(x), ptr(n0.weight), ptr(n0.bias), float(n0.eps),
                 ptr(st.n), ptr(st.npos), s)
        for li, layer in enumerate(layers):
            sa, ca, ff = layer.tgt_self_attn, layer.tgt_src_cross_attn, layer.ff
            sub, csub = sa.sublayer, ca.sublayer
            f0, f2 = ff.sublayer[0], ff.sublayer[2]
            if embed and li == 0:
                call("retr_dec_self_heads_embed", ptr(st.tok), ptr(emb.word_embeddings.weight),
                     ptr(emb.LayerNorm.weight), ptr(emb.LayerNorm.bias),
                     float(emb.LayerNorm.eps), R, C, H, ptr(W(sub.in_proj_weight)),
                     ptr(sub.in_proj_bias), ptr(st.kc[li]), ptr(st.vc[li]), i, T, anc,
                     ptr(W(sub.out_proj.weight)), ptr(st.hslab), ptr(n0.weight), ptr(n0.bias),
                     float(n0.eps), ptr(qp), ptr(x), s)
            elif fold and li > 0:
                pf2 = layers[li - 1].ff.sublayer[2]
                call("retr_dec_self_heads_mr", None, None, R, C, H,
                     ptr(W(sub.in_proj_weight)), ptr(sub.in_proj_bias), ptr(st.kc[li]),
                     ptr(st.vc[li]), i, T, anc, ptr(W(sub.out_proj.weight)), ptr(st.hslab),
                     ptr(x), ptr(st.slabs), F // hb, ptr(pf2.bias), ptr(sa.norm.weight),
                     ptr(sa.norm.bias), float(sa.norm.eps), ptr(qp), ptr(xa), rbs, s)
                x, xa = xa, x
            else:
                call("retr_dec_self_heads_mr", ptr(st.n), ptr(st.npos), R, C, H,
                     ptr(W(sub.in_proj_weight)), ptr(sub.in_proj_bias), ptr(st.kc[li]),
                     ptr(st.vc[li]), i, T, anc, ptr(W(sub.out_proj.weight)), ptr(st.hslab),
                     None, None, 0, None, None, None, 0.0, None, None, rbs, s)
            call("retr_dec_cross_heads_mr", ptr(st.hslab), ptr(x), ptr(sub.out_proj.bias),
                 ptr(xa), R, C, H, ptr(ca.norm.weight), ptr(ca.norm.bias), float(ca.norm.eps),
                 ptr(qp), ptr(W(csub.in_proj_weight)), ptr(csub.in_proj_bias), ptr(st.kx[li]),
                 ptr(st.vx[li]), S, st.K, ptr(st.kpm), ptr(W(csub.out_proj.weight)),
                 ptr(st.hslab2), rbx, s)
            x, xa = xa, x
            if fold:
                call("retr_dec_ffn_ln128" if hb == 128 else "retr_dec_ffn_ln64", ptr(x),
                     ptr(st.hslab2), H, ptr(csub.out_proj.bias),
                     ptr(ff.norm.weight), ptr(ff.norm.bias), float(ff.norm.eps), ptr(xa), R, C,
                     ptr(W(f0.weight)), ptr(f0.bias), ptr(W(f2.weight)), F, ptr(st.slabs), s)
                x, xa = xa, x
                if li + 1 == len(layers):
                    nx = tr.decoder.norm
                    call("retr_dec_rows", ptr(x), ptr(st.slabs), F // hb, ptr(f2.bias), R, C,
                         ptr(xa), ptr(nx.weight), ptr(nx.bias), float(nx.eps), None, ptr(st.n),
                         None, s)
                    x, xa = xa, x
                continue
            if DEC_FFN_LN and R <= 64:
                # (every FFN block re-derives its 16 rows' LayerNorm: beyond 64 rows the
                # repeated slab reads cost more than the separate launch saves)
                call("retr_dec_ffn_ln", ptr(x), ptr(st.hslab2), H, ptr(csub.out_proj.bias),
                     ptr(ff.norm.weight), ptr(ff.norm.bias), float(ff.norm.eps), ptr(xa), R, C,
                     ptr(W(f0.weight)), ptr(f0.bias), ptr(W(f2.weight)), F, ptr(st.slabs), s)
            else:
                call("retr_dec_rows", ptr(x), ptr(st.hslab2), H, ptr(csub.out_proj.bias), R, C,
                     ptr(xa), ptr(ff.norm.weight), ptr(ff.norm.bias), float(ff.norm.eps), None,
                     ptr(st.o), None, s)
                call("retr_dec_ffn", ptr(st.o), R, C, ptr(W(f0.weight)), ptr(f0.bias),
                     ptr(W(f2.weight)), F, ptr(st.slabs), s)
            x, xa = xa, x
            if li + 1 < len(layers):
                nx, npos = layers[li + 1].tgt_self_attn.norm, ptr(st.npos)
            else:
                nx, npos = tr.decoder.norm, None
            call("retr_dec_rows", ptr(x), ptr(st.slabs), nslab, ptr(f2.bias), R, C, ptr(xa),
                 ptr(nx.weight), ptr(nx.bias), float(nx.eps), ptr(qp) if npos else None,
                 ptr(st.n), npos, s)
            x, xa = xa, x
        l1, l2, l3 = model.mlp.layers
        V = l3.weight.shape[0]
        H1 = l1.weight.shape[0]
        w1, w2 = W(l1.weight), W(l2.weight)
        if DEC_HEAD_SKINNY and R <= 512 and C % 32 == 0 and H1 % 32 == 0:
            # the head's first two layers on the 16 x 16-tile decode linear (128 blocks each)
            call("retr_dec_linear_bf16", ptr(st.n), C, ptr(w1), C, ptr(l1.bias), ptr(st.h1),
                 st.h1.stride(0), R, H1, C, 1, s)
            call("retr_dec_linear_bf16", ptr(st.h1), st.h1.stride(0), ptr(w2), w2.stride(0),
                 ptr(l2.bias), ptr(st.h2), st.h2.stride(0), R, w2.shape[0], H1, 1, s)
        else:
            call("retr_dec_gemm", ptr(st.n), None, R, C, ptr(w1), ptr(l1.bias), H1,
                 ptr(st.h1), H1, 0, None, 0, 0, None, 0, 0, H1, 1, s)
            k_linear_fwd(st.h1, w2, l2.bias.detach(), st.h2, relu=1)
        k_linear_fwd(st.h2, ops.WEIGHTS.get(l3.weight, cd, rows=st.Vp), st.head_bias, st.logits)
        self._select(st, i, V, eos_token, s)

    def _select(self, st, i, V, eos_token, s):
        """Greedy: first-index argmax + the reference's finished/early-exit bookkeeping (a row
        group of a split batch writes every column: _call_split ends the batch)."""
        cd = self.cdtype
        call("retr_greedy_select2", dcode(cd), ptr(st.logits), st.Vp, st.B, V, ptr(st.am_ws),
             st.T, i, int(eos_token), ptr(st.pred), ptr(st.caption), ptr(st.finished),
             ptr(st.done), ptr(st.tok), int(st.write_all), s)

    # -- state handling (overridden by IncrementalBeam) --------------------------------------
    def _new_state(self, B, S, T, C, F, L, V, cd, dev):
        return _DecodeState(B, S, T, C, F, L, V, cd, dev)

    def _reset(self, st, bos_token):
        st.caption.zero_()
        st.caption[:, 0] = bos_token
        st.tok.fill_(bos_token)
        st.finished.zero_()
        st.done.fill_(-1)

    def _result(self, st):
        return st.caption.clone()

    def _state(self, key, B, S, T, C, dev):
        st = self.states.get(key)
        if st is None:
            layers = list(self.tr.decoder.layers)
            st = self._new_state(B, S, T, C, layers[0].ff.sublayer[0].weight.shape[0],
                                 len(layers), self.model.mlp.layers[2].weight.shape[0],
                                 self.cdtype, dev)
            self.states[key] = st
        return st

    def _memory_kv(self, st, mem, mem_pos, kpm):
        """The cross-attention K/V of every decoder layer, once per batch, into the static
        buffers of ``st`` (mem / mem_pos: its rows' memory tokens)."""
        cd = self.cdtype
        C = mem.shape[1]
        for li, layer in enumerate(self.tr.decoder.layers):
            sub = layer.tgt_src_cross_attn.sublayer
            w = ops.WEIGHTS.get(sub.in_proj_weight, cd)
            b = sub.in_proj_bias.detach()
            k_linear_fwd(mem_pos, w[C:2 * C], b[C:2 * C], st.kx[li])
            k_linear_fwd(mem, w[2 * C:], b[2 * C:], st.vx[li])
        st.kpm.copy_(kpm)

    def _split(self, B):
        """Row groups of a batch decoded concurrently (DEC_SPLIT)."""
        n = DEC_SPLIT
        if self.beam or not self.use_graphs or n < 2 or B % n or B // n < DEC_SPLIT_MIN_ROWS:
            return 1
        return n

    @torch.no_grad()
    def __call__(self, samples, max_len, bos_token, eos_token, poll=8):
        """samples: the model's memory inputs (a NestedTensor for Caption; the argument list of
        CaptionLoc / CaptionGlobalLoc before the caption), as passed to ``greedy``."""
        model, tr, cd = self.model, self.tr, self.cdtype
        if not isinstance(samples, (list, tuple)):
            samples = [samples]
        src, mask, B, S = model.memory_tokens(*samples)
        kpm = mask.reshape(B, S).contiguous().view(torch.uint8)
        mem, mem_pos, _ = tr.encode(src, B, S, kpm, cd)
        qpos_w = tr.embeddings.position_embeddings.weight
        T = max_len
        if T != qpos_w.shape[0]:
            raise RuntimeError(f"The size of tensor a ({T}) must match the size of tensor b "
                               f"({qpos_w.shape[0]}) at non-singleton dimension 0")
        C = mem.shape[1]
        n = self._split(B)
        if n > 1:
            return self._call_split(n, mem, mem_pos, kpm, B, S, T, C, bos_token, eos_token)
        key = (type(self).__name__, self.K, B, S, T, cd, int(eos_token), bool(self.fused))
        st = self._state(key, B, S, T, C, mem.device)
        self._memory_kv(st, mem, mem_pos, kpm)
        self._reset(st, bos_token)
        sig = self._signature()
        if st.signature != sig:
            st.head_bias = ops._pad_vec(model.mlp.layers[2].bias, st.Vp)
            st.graphs = None
        if self.use_graphs and st.graphs is None:
            # warm once eagerly (kernel attributes, weight copies), then capture every step
            self._step(st, 0, eos_token)
            torch.cuda.synchronize()
            self._reset(st, bos_token)
            # DEC_GRAPH_STEPS consecutive steps per graph (one replay launch each, the host
            # polls `done` between graphs)
            graphs = []
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for i0 in range(0, T - 1, DEC_GRAPH_STEPS):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=side):
                        for i in range(i0, min(i0 + DEC_GRAPH_STEPS, T - 1)):
                            self._step(st, i, eos_token)
                    graphs.append(g)
            torch.cuda.current_stream().wait_stream(side)
            st.graphs = graphs
        st.signature = sig
        if self.use_graphs:
            for g in st.graphs:
                g.replay()
                if int(st.done.item()) >= 0:
                    break
        else:
            for i in range(T - 1):
                self._step(st, i, eos_token)
                if (i + 1) % poll == 0 and int(st.done.item()) >= 0:
                    break
        return self._result(st)

    def _call_split(self, n, mem, mem_pos, kpm, B, S, T, C, bos_token, eos_token):
        """The batch as n independent row groups (their own state, captured on n streams of
        ONE graph per DEC_GRAPH_STEPS steps, so the groups' latency-bound step kernels overlap
        on the GPU).  Rows never interact in a step, so every id is the unsplit decoder's: each
        group writes every column (retr_greedy_select2 write_all) and records its first
        all-finished step; the batch ends at the last group's -- the reference's exit
        (decode.py:77-79: all rows finished) -- and the columns after it are cleared, as the
        unsplit step leaves them."""
        cd = self.cdtype
        Bh = B // n
        base = (type(self).__name__, self.K, Bh, S, T, cd, int(eos_token), bool(self.fused))
        sts = [self._state(base + ("split", h, n), Bh, S, T, C, mem.device) for h in range(n)]
        for h, st in enumerate(sts):
            st.write_all = True
            rows = slice(h * Bh * S, (h + 1) * Bh * S)
            self._memory_kv(st, mem[rows], mem_pos[rows], kpm[h * Bh:(h + 1) * Bh])
            self._reset(st, bos_token)
        sig = self._signature()
        st0 = sts[0]
        if st0.signature != sig:
            for st in sts:
                st.head_bias = ops._pad_vec(self.model.mlp.layers[2].bias, st.Vp)
            st0.graphs = None
        if st0.graphs is None:
            for st in sts:                  # warm once eagerly (attributes, weight copies)
                self._step(st, 0, eos_token)
            torch.cuda.synchronize()
            for st in sts:
                self._reset(st, bos_token)
            graphs = []
            side = torch.cuda.Stream()
            lanes = [torch.cuda.Stream() for _ in range(n - 1)]
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for i0 in range(0, T - 1, DEC_GRAPH_STEPS):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=side):
                        for ln in lanes:
                            ln.wait_stream(side)
                        for h, st in enumerate(sts):
                            with torch.cuda.stream(side if h == 0 else lanes[h - 1]):
                                for i in range(i0, min(i0 + DEC_GRAPH_STEPS, T - 1)):
                                    self._step(st, i, eos_token)
                        for ln in lanes:
                            side.wait_stream(ln)
                    graphs.append(g)
            torch.cuda.current_stream().wait_stream(side)
            st0.graphs = graphs
        st0.signature = sig
        dones = torch.stack([st.done for st in sts])
        for g in st0.graphs:
            g.replay()
            torch.stack([st.done for st in sts], out=dones)
            if int(dones.min().item()) >= 0:
                break
        ids = torch.cat([self._result(st) for st in sts])
        if int(dones.min().item()) >= 0:
            ids[:, int(dones.max().item()) + 1:] = 0
        return ids


class IncrementalBeam(IncrementalGreedy):
    """KV-cache beam search (new capability: the reference decodes greedily only,
    eval_utils/decode.py:53-81).  K beams per image run as B*K decoder rows; per step
    ``retr_topk_rows`` gives every row its K best tokens and log-softmax values and
    ``retr_beam_select`` keeps the K best of (finished beams: their score and argmax
    continuation; others: score + log p of each of their K tokens), reorders the token history
    and the cache-ancestry table (csrc/beam.hip), so the K/V caches are never copied.  The loop
    ends like greedy's: at the first step after which every beam of every image has emitted
    EOS, whose column is not written.  Result: each image's highest-scoring beam (optionally
    length-normalised), in greedy's caption format.  With K = 1 it is greedy, token for token.
    """

    beam = True

    def __init__(self, model, beam_size=5, use_graphs=True, length_penalty=0.0):
        super().__init__(model, use_graphs)
        if not 1 <= beam_size <= 8:
            raise ValueError(f"beam_size must be in [1, 8], got {beam_size}")
        self.K = beam_size
        self.length_penalty = float(length_penalty)
        self.last_scores = None

    def _new_state(self, B, S, T, C, F, L, V, cd, dev):
        st = _DecodeState(B, S, T, C, F, L, V, cd, dev, K=self.K)
        if self.K == 1:
            st.init_beam(dev)
        return st

    def _reset(self, st, bos_token):
        st.hist.zero_()
        st.hist[:, 0] = bos_token
        st.anc.copy_(torch.arange(st.R, dtype=torch.int32, device=st.anc.device)[:, None]
                     .expand(st.R, st.T))
        st.scores.zero_()
        st.tok.fill_(bos_token)
        st.finished.zero_()
        st.item_done.zero_()
        st.done.fill_(-1)

    def __call__(self, samples, max_len, bos_token, eos_token, poll=8):
        self._eos = int(eos_token)
        return super().__call__(samples, max_len, bos_token, eos_token, poll)

    def _select(self, st, i, V, eos_token, s):
        call("retr_topk_rows", dcode(self.cdtype), ptr(st.logits), st.Vp, st.R, V, st.K,
             ptr(st.cand_tok), ptr(st.cand_lp), s)
        call("retr_beam_select", ptr(st.cand_tok), ptr(st.cand_lp), st.B, st.K, i, st.T,
             int(eos_token), ptr(st.scores), ptr(st.finished), ptr(st.hist), ptr(st.anc),
             ptr(st.tok), ptr(st.item_done), ptr(st.done), s)

    def _result(self, st):
        B, K, T = st.B, st.K, st.T
        done = int(st.done.item())
        hist = st.hist.view(B, K, T)
        scores = st.scores.view(B, K)
        if self.length_penalty:
            # GNMT length normalisation; length = tokens after BOS up to the first EOS
            is_eos = hist[..., 1:] == self._eos
            first = is_eos.int().argmax(-1) + 1
            length = torch.where(is_eos.any(-1), first, torch.full_like(first, T - 1)).float()
            scores = scores / ((5.0 + length) / 6.0) ** self.length_penalty
        best = scores.argmax(-1)
        cap = hist[torch.arange(B, device=hist.device), best].clone()
        if done >= 0:
            cap[:, done + 1:] = 0
        self.last_scores = scores.gather(1, best[:, None])[:, 0]
        return cap
def _full_forward_greedy(samples, model, max_len, bos_token, eos_token, device):
    """The reference algorithm (decode.py:59-81) on the MI355X kernels: one full model forward
    per step.  Used when the model is in training mode (dropout active) and for parity tests."""
    caption, cap_mask = create_caption_and_mask(bos_token, max_len, samples[0].shape[0])
    samples = [s.to(device) for s in samples]
    caption = caption.to(device)
    cap_mask = cap_mask.to(device)
    finished = torch.zeros(caption.shape[0], dtype=torch.bool, device=device)
    for i in range(max_len - 1):
        predictions = model(*samples, caption, cap_mask)
        pid = ops.argmax_rows(predictions[:, i, :])
        finished = torch.logical_or(pid == eos_token, finished)
        if bool(finished.all()):
            return caption
        caption[:, i + 1] = pid
        cap_mask[:, i + 1] = False
    return caption


def greedy(samples, model, max_len=20, device="auto", bos_token=1, eos_token=2):
    """greedy decoding for a batch of samples (decode.py:53-81 contract)."""
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    samples = [s.to(device) for s in samples]
    if model.training or not hasattr(model, "memory_tokens"):
        return _full_forward_greedy(samples, model, max_len, bos_token, eos_token, device)
    return IncrementalGreedy(model)(samples, max_len, bos_token, eos_token)


def beam_search(samples, model, max_len=20, beam_size=5, device="auto", bos_token=1,
                eos_token=2, length_penalty=0.0):
    """Beam-search decoding for a batch of samples (new; the reference has greedy only).  Same
    inputs and caption format as ``greedy``; ``beam_size=1`` returns exactly greedy's ids."""
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    samples = [s.to(device) for s in samples]
    if model.training:
        raise RuntimeError("beam_search runs in eval mode (model.eval())")
    return IncrementalBeam(model, beam_size, length_penalty=length_penalty)(
        samples, max_len, bos_token, eos_token)


def beam_decoding(samples, model, tokenizer, max_len=20, beam_size=5, clean=True, pad_token=0,
                  bos_token=1, eos_token=2, device="auto", length_penalty=0.0):
    """greedy_decoding's wrapper (decode.py:112-128) around ``beam_search``."""
    caption_idx = beam_search(samples, model, max_len=max_len, beam_size=beam_size,
                              device=device, bos_token=bos_token, eos_token=eos_token,
                              length_penalty=length_penalty)
    caption_idx = caption_idx.cpu().detach().numpy().tolist()
    pruned = prune_cap_ids(caption_idx, clean=clean, pad_token=pad_token, bos_token=bos_token,
                           eos_token=eos_token)
    return idx2sents(pruned, tokenizer)


def greedy_reference_algorithm(samples, model, max_len, bos_token=1, eos_token=2,
                               device="cuda"):
    """Full-recompute greedy (127 forwards), exposed for parity checks against ``greedy``."""
    with torch.no_grad():
        return _full_forward_greedy(list(samples), model, max_len, bos_token, eos_token, device)


def prune_cap_ids(idx_seqs, clean=True, pad_token=0, bos_token=1, eos_token=2):
    """cut off index sequences; optionally clean <PAD>, <BOS>, <EOS> (decode.py:84-101)."""
    results = []
    for seq in idx_seqs:
        pruned = []
        for idx in seq:
            pruned.append(idx)
            if idx == eos_token:
                break
        if clean:
            pruned = [i for i in pruned if i not in (pad_token, bos_token, eos_token)]
        results.append(pruned)
    return results


def idx2sents(idx_seqs, tokenizer, skip_special_tokens=True):
    return tokenizer.batch_decode(idx_seqs, skip_special_tokens=skip_special_tokens)


def greedy_decoding(samples, model, tokenizer, max_len=20, clean=True, pad_token=0, bos_token=1,
                    eos_token=2, device="auto"):
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    caption_idx = greedy(samples, model, max_len=max_len, bos_token=bos_token,
                         eos_token=eos_token, device=device)
    caption_idx = caption_idx.cpu().detach().numpy().tolist()
    pruned = prune_cap_ids(caption_idx, clean=clean, pad_token=pad_token, bos_token=bos_token,
                           eos_token=eos_token)
    return idx2sents(pruned, tokenizer)


def greedy_single(model, image, tokenizer, start_token, end_token, max_pos_embeddings):
    """greedy decoding for a single image (decode.py:30-50)."""
    caption, cap_mask = create_caption_and_mask(start_token, max_pos_embeddings)
    dev = image.tensors.device if hasattr(image, "tensors") else image.device
    caption, cap_mask = caption.to(dev), cap_mask.to(dev)
    with torch.no_grad():
        model.eval()
        for i in range(max_pos_embeddings - 1):
            predictions = model(image, caption, cap_mask)
            predicted_id = ops.argmax_rows(predictions[:, i, :])
            if int(predicted_id[0]) == end_token:
                break
            caption[:, i + 1] = predicted_id[0]
            cap_mask[:, i + 1] = False
    return tokenizer.decode(caption[0], skip_special_tokens=True)


def greedy_with_att(model, sample, tokenizer, start_token=1, end_token=2, max_pos_embeddings=128,
                    return_raw=True, device="auto"):
    """single image, collects attention maps per step (decode.py:131-167)."""
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    caption, cap_mask = create_caption_and_mask(start_token, max_pos_embeddings)
    sample = [s.to(device) for s in sample]
    caption, cap_mask = caption.to(device), cap_mask.to(device)
    atts = []
    with torch.no_grad():
        model.eval()
        for i in range(max_pos_embeddings - 1):
            predictions, att = model(*sample, caption, cap_mask, return_attention=True)
            predicted_id = ops.argmax_rows(predictions[:, i, :])
            caption[:, i + 1] = predicted_id[0]
            cap_mask[:, i + 1] = False
            atts.append(att)
            if int(predicted_id[0]) == end_token:
                break
    token_ids = caption[0][~cap_mask[0]][1:]
    if return_raw:
        return token_ids, atts
    return tokenizer.decode(token_ids, skip_special_tokens=True), atts
