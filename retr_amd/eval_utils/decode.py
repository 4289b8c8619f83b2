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
from .._lib import call, ptr
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


class _DecodeState:
    """Static device buffers (and captured per-step hipGraphs) for one (B, S, T) shape."""

    def __init__(self, B, S, T, C, F, n_layers, V, cd, dev):
        f32 = torch.float32
        self.B, self.S, self.T = B, S, T
        self.kx = [torch.empty(B * S, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.vx = [torch.empty(B * S, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.kc = [torch.zeros(B * T, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.vc = [torch.zeros(B * T, C, dtype=cd, device=dev) for _ in range(n_layers)]
        self.kpm = torch.zeros(B, S, dtype=torch.uint8, device=dev)
        self.caption = torch.zeros(B, T, dtype=torch.long, device=dev)
        self.tok = torch.zeros(B, dtype=torch.long, device=dev)
        self.finished = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.done = torch.full((1,), -1, dtype=torch.int32, device=dev)
        self.y = torch.empty(B, C, dtype=f32, device=dev)
        self.y2 = torch.empty_like(self.y)
        self.n = torch.empty(B, C, dtype=cd, device=dev)
        self.npos = torch.empty_like(self.n)
        self.q = torch.empty_like(self.n)
        self.o = torch.empty_like(self.n)
        self.mean = torch.empty(B, dtype=f32, device=dev)
        self.rstd = torch.empty_like(self.mean)
        self.ffh = torch.empty(B, F, dtype=cd, device=dev)
        self.h1 = torch.empty(B, 512, dtype=cd, device=dev)
        self.h2 = torch.empty(B, 512, dtype=cd, device=dev)
        self.Vp = (V + 63) // 64 * 64
        self.logits = torch.empty(B, self.Vp, dtype=cd, device=dev)
        self.pred = torch.empty(B, dtype=torch.long, device=dev)
        self.head_bias = None
        self.graphs = None
        self.signature = None


class IncrementalGreedy:
    """KV-cache greedy decoder over a ``Caption`` model (eval mode semantics).  The T-1 decode
    steps are captured once per (shape, weights) as hipGraphs and replayed per batch."""

    def __init__(self, model, use_graphs=True):
        self.model = model
        self.tr = model.transformer
        self.cdtype = model.cdtype
        self.use_graphs = use_graphs
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

    def _step(self, st, i, eos_token):
        """Kernels of decode step i (reads token i, writes caption column i+1)."""
        model, tr, cd = self.model, self.tr, self.cdtype
        B, S, T = st.B, st.S, st.T
        C = st.n.shape[1]
        layers = list(tr.decoder.layers)
        H = layers[0].tgt_self_attn.sublayer.num_heads
        hd = C // H
        emb = tr.embeddings
        qp = emb.position_embeddings.weight.detach()[i]
        s = _st()
        y, y2 = st.y, st.y2
        call("retr_embed_ln_fwd", ptr(st.tok), B, 1, C, ptr(emb.word_embeddings.weight), ptr(qp),
             ptr(emb.LayerNorm.weight), ptr(emb.LayerNorm.bias), float(emb.LayerNorm.eps), 0.0, 0,
             ptr(y), ptr(st.mean), ptr(st.rstd), s)
        for li, layer in enumerate(layers):
            sa = layer.tgt_self_attn
            sub = sa.sublayer
            w = ops.WEIGHTS.get(sub.in_proj_weight, cd)
            b = sub.in_proj_bias.detach()
            self._ln(y, sa.norm, y=st.n, y2=st.npos, pos=qp)
            k_linear_fwd(st.npos, w[:C], b[:C], st.q)
            k_linear_fwd(st.npos, w[C:2 * C], b[C:2 * C], st.kc[li][i::T])
            k_linear_fwd(st.n, w[2 * C:], b[2 * C:], st.vc[li][i::T])
            call("retr_attention_decode", dcode(cd), ptr(st.q), C, ptr(st.kc[li]), C,
                 ptr(st.vc[li]), C, ptr(st.o), C, B, H, i + 1, T, hd, None, s)
            k_linear_fwd(st.o, ops.WEIGHTS.get(sub.out_proj.weight, cd),
                         sub.out_proj.bias.detach(), y2, res=y)
            y, y2 = y2, y
            ca = layer.tgt_src_cross_attn
            sub = ca.sublayer
            w = ops.WEIGHTS.get(sub.in_proj_weight, cd)
            b = sub.in_proj_bias.detach()
            self._ln(y, ca.norm, y2=st.npos, pos=qp)
            k_linear_fwd(st.npos, w[:C], b[:C], st.q)
            call("retr_attention_decode", dcode(cd), ptr(st.q), C, ptr(st.kx[li]), C,
                 ptr(st.vx[li]), C, ptr(st.o), C, B, H, S, S, hd, ptr(st.kpm), s)
            k_linear_fwd(st.o, ops.WEIGHTS.get(sub.out_proj.weight, cd),
                         sub.out_proj.bias.detach(), y2, res=y)
            y, y2 = y2, y
            ff = layer.ff
            self._ln(y, ff.norm, y=st.n)
            f0, f2 = ff.sublayer[0], ff.sublayer[2]
            k_linear_fwd(st.n, ops.WEIGHTS.get(f0.weight, cd), f0.bias.detach(), st.ffh, relu=1)
            k_linear_fwd(st.ffh, ops.WEIGHTS.get(f2.weight, cd), f2.bias.detach(), y2, res=y)
            y, y2 = y2, y
        l1, l2, l3 = model.mlp.layers
        V = l3.weight.shape[0]
        self._ln(y, tr.decoder.norm, y=st.n)
        k_linear_fwd(st.n, ops.WEIGHTS.get(l1.weight, cd), l1.bias.detach(), st.h1, relu=1)
        k_linear_fwd(st.h1, ops.WEIGHTS.get(l2.weight, cd), l2.bias.detach(), st.h2, relu=1)
        k_linear_fwd(st.h2, ops.WEIGHTS.get(l3.weight, cd, rows=st.Vp),
                     st.head_bias, st.logits)
        call("retr_argmax_rows", dcode(cd), ptr(st.logits), st.Vp, B, V, ptr(st.pred), s)
        call("retr_greedy_update", ptr(st.pred), B, T, i, int(eos_token), ptr(st.caption),
             ptr(st.finished), ptr(st.done), ptr(st.tok), s)

    @torch.no_grad()
    def __call__(self, samples, max_len, bos_token, eos_token, poll=8):
        model, tr, cd = self.model, self.tr, self.cdtype
        src, mask, B, S = model.encode_image(samples)
        kpm = mask.reshape(B, S).contiguous().view(torch.uint8)
        mem, mem_pos, _ = tr.encode(src, B, S, kpm, cd)
        qpos_w = tr.embeddings.position_embeddings.weight
        T = max_len
        if T != qpos_w.shape[0]:
            raise RuntimeError(f"The size of tensor a ({T}) must match the size of tensor b "
                               f"({qpos_w.shape[0]}) at non-singleton dimension 0")
        C = mem.shape[1]
        layers = list(tr.decoder.layers)
        key = (B, S, T, cd, int(eos_token))
        st = self.states.get(key)
        if st is None:
            st = _DecodeState(B, S, T, C, layers[0].ff.sublayer[0].weight.shape[0], len(layers),
                              model.mlp.layers[2].weight.shape[0], cd, mem.device)
            self.states[key] = st
        # cross-attention K/V of every decoder layer, once per batch, into the static buffers
        for li, layer in enumerate(layers):
            sub = layer.tgt_src_cross_attn.sublayer
            w = ops.WEIGHTS.get(sub.in_proj_weight, cd)
            b = sub.in_proj_bias.detach()
            k_linear_fwd(mem_pos, w[C:2 * C], b[C:2 * C], st.kx[li])
            k_linear_fwd(mem, w[2 * C:], b[2 * C:], st.vx[li])
        st.kpm.copy_(kpm)
        st.caption.zero_()
        st.caption[:, 0] = bos_token
        st.tok.fill_(bos_token)
        st.finished.zero_()
        st.done.fill_(-1)
        sig = self._signature()
        if st.signature != sig:
            st.head_bias = ops._pad_vec(model.mlp.layers[2].bias, st.Vp)
            st.graphs = None
        if self.use_graphs and st.graphs is None:
            # warm once eagerly (kernel attributes, weight copies), then capture every step
            self._step(st, 0, eos_token)
            torch.cuda.synchronize()
            st.caption.zero_()
            st.caption[:, 0] = bos_token
            st.tok.fill_(bos_token)
            st.finished.zero_()
            st.done.fill_(-1)
            graphs = []
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for i in range(T - 1):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=side):
                        self._step(st, i, eos_token)
                    graphs.append(g)
            torch.cuda.current_stream().wait_stream(side)
            st.graphs = graphs
        st.signature = sig
        for i in range(T - 1):
            if self.use_graphs:
                st.graphs[i].replay()
            else:
                self._step(st, i, eos_token)
            if (i + 1) % poll == 0 and int(st.done.item()) >= 0:
                break
        return st.caption.clone()


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
    if model.training or not hasattr(model, "encode_image"):
        return _full_forward_greedy(samples, model, max_len, bos_token, eos_token, device)
    return IncrementalGreedy(model)(samples[0], max_len, bos_token, eos_token)


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
