"""Functional fp32 CPU restatement of the RE⫶TR hot path (TEST INFRASTRUCTURE ONLY).

Every function cites the reference file:line it restates.  It runs on a plain ``state_dict``
(same keys as the reference ``Caption`` model) so it needs no reference import at run time and
travels to the GPU box with the tests.  Dropout is the identity here (parity is defined with
``dropout=0``/``.eval()``, SURVEY.md §7 hard part (iv)).

Pinned against the reference itself by ``tests/golden/make_golden.py`` (vectors in
``tests/golden/*.npz``; see ``tests/test_oracle.py``).
"""
import math

import torch
import torch.nn.functional as F

# ---------------------------------------------------------------------------------------------
# backbone  (models/backbone.py + torchvision resnet semantics)
# ---------------------------------------------------------------------------------------------

_ARCH = {"resnet18": ("basic", [2, 2, 2, 2]), "resnet34": ("basic", [3, 4, 6, 3]),
         "resnet50": ("bottleneck", [3, 4, 6, 3]), "resnet101": ("bottleneck", [3, 4, 23, 3])}


def resnet_plan(name, dilation):
    """Per-block (prefix, kind, inplanes, planes, stride, dilation, has_downsample) list.
    torchvision ``_make_layer`` semantics with ``replace_stride_with_dilation=[F,F,dilation]``
    (models/backbone.py:89-91)."""
    kind, layers = _ARCH[name.lower()]
    exp = 1 if kind == "basic" else 4
    inplanes, cur_dil, plan = 64, 1, []
    for li, (planes, nblk, stride, dil_flag) in enumerate(
            zip([64, 128, 256, 512], layers, [1, 2, 2, 2], [False, False, False, dilation])):
        prev_dil = cur_dil
        if dil_flag:
            cur_dil *= stride
            stride = 1
        ds = stride != 1 or inplanes != planes * exp
        for bi in range(nblk):
            d = prev_dil if bi == 0 else cur_dil
            if kind == "basic" and d > 1:
                raise NotImplementedError("Dilation > 1 not supported in BasicBlock")
            plan.append((f"layer{li + 1}.{bi}", kind, inplanes, planes,
                         stride if bi == 0 else 1, d, ds and bi == 0))
            inplanes = planes * exp
    return plan


def frozen_bn(x, sd, p):
    """models/backbone.py:41-51 (scale/bias recomputed in fp32 every call, eps 1e-5)."""
    w = sd[p + ".weight"].reshape(1, -1, 1, 1)
    b = sd[p + ".bias"].reshape(1, -1, 1, 1)
    rv = sd[p + ".running_var"].reshape(1, -1, 1, 1)
    rm = sd[p + ".running_mean"].reshape(1, -1, 1, 1)
    scale = w * (rv + 1e-5).rsqrt()
    bias = b - rm * scale
    return x * scale + bias


def resnet_body(x, sd, name, dilation, pre="backbone.body."):
    """IntermediateLayerGetter(resnet, {'layer4': '0'}) (models/backbone.py:65,69)."""
    x = F.conv2d(x, sd[pre + "conv1.weight"], stride=2, padding=3)
    x = F.relu(frozen_bn(x, sd, pre + "bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for (p, kind, _cin, _planes, stride, dil, ds) in resnet_plan(name, dilation):
        q = pre + p + "."
        idt = x
        if ds:
            idt = frozen_bn(F.conv2d(x, sd[q + "downsample.0.weight"], stride=stride), sd,
                            q + "downsample.1")
        if kind == "basic":
            o = F.relu(frozen_bn(F.conv2d(x, sd[q + "conv1.weight"], stride=stride, padding=1),
                                 sd, q + "bn1"))
            o = frozen_bn(F.conv2d(o, sd[q + "conv2.weight"], padding=1), sd, q + "bn2")
        else:
            o = F.relu(frozen_bn(F.conv2d(x, sd[q + "conv1.weight"]), sd, q + "bn1"))
            o = F.relu(frozen_bn(F.conv2d(o, sd[q + "conv2.weight"], stride=stride, padding=dil,
                                          dilation=dil), sd, q + "bn2"))
            o = frozen_bn(F.conv2d(o, sd[q + "conv3.weight"]), sd, q + "bn3")
        x = F.relu(o + idt)
    return x


def mask_to_features(mask, hw):
    """models/backbone.py:75 — nearest interpolation of the pixel mask to the feature grid."""
    return F.interpolate(mask[None].float(), size=hw).to(torch.bool)[0]


# ---------------------------------------------------------------------------------------------
# transformer  (models/ConcatTransformer.py, models/transformer_modules.py, torch MHA)
# ---------------------------------------------------------------------------------------------

def sine_table(d_model, max_len=1024):
    """models/position_encoding.py:16-22 -> buffer ``pe`` [max_len, 1, d_model]."""
    position = torch.arange(max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
    pe = torch.zeros(max_len, 1, d_model)
    pe[:, 0, 0::2] = torch.sin(position * div_term)
    pe[:, 0, 1::2] = torch.cos(position * div_term)
    return pe


def causal_mask(sz):
    """models/utils.py:50-57: float mask, 0 on/below the diagonal, -inf above."""
    m = (torch.triu(torch.ones(sz, sz)) == 1).transpose(0, 1)
    return m.float().masked_fill(m == 0, float("-inf")).masked_fill(m == 1, 0.0)


def mha(query, key, value, sd, p, nhead, key_padding_mask=None, attn_mask=None):
    """``nn.MultiheadAttention.forward`` -> ``F.multi_head_attention_forward`` need_weights path
    (torch/nn/functional.py:5785-5850 in-projection, :6553-6567 mask merge, :6576-6613 core).
    Inputs are seq-first [L, B, C].  Returns (out [Lq,B,C], head-averaged P [B,Lq,Lk])."""
    lq, bsz, c = query.shape
    lk = key.shape[0]
    hd = c // nhead
    w, b = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
    wq, wk, wv = w.chunk(3)
    bq, bk, bv = b.chunk(3)
    q = F.linear(query, wq, bq)
    k = F.linear(key, wk, bk)
    v = F.linear(value, wv, bv)
    q = q.view(lq, bsz * nhead, hd).transpose(0, 1)
    k = k.view(lk, bsz * nhead, hd).transpose(0, 1)
    v = v.view(lk, bsz * nhead, hd).transpose(0, 1)
    mask = None
    if attn_mask is not None:
        mask = attn_mask.unsqueeze(0)
    if key_padding_mask is not None:
        kpm = torch.zeros(key_padding_mask.shape, dtype=q.dtype).masked_fill_(
            key_padding_mask, float("-inf"))
        kpm = kpm.view(bsz, 1, 1, lk).expand(-1, nhead, -1, -1).reshape(bsz * nhead, 1, lk)
        mask = kpm if mask is None else mask + kpm
    qs = q * math.sqrt(1.0 / float(hd))
    if mask is not None:
        att = torch.baddbmm(mask, qs, k.transpose(-2, -1))
    else:
        att = torch.bmm(qs, k.transpose(-2, -1))
    att = F.softmax(att, dim=-1)
    out = torch.bmm(att, v)
    out = out.transpose(0, 1).contiguous().view(lq * bsz, c)
    out = F.linear(out, sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"]).view(lq, bsz, c)
    return out, att.view(bsz, nhead, lq, lk).mean(dim=1)


def layer_norm(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def feed_forward(x, sd, p):
    """models/transformer_modules.py:6-11 (Linear -> ReLU -> Linear)."""
    return F.linear(F.relu(F.linear(x, sd[p + ".0.weight"], sd[p + ".0.bias"])),
                    sd[p + ".2.weight"], sd[p + ".2.bias"])


def encoder_layer(x, sd, p, nhead, pos, kpm):
    """TransformerEncoderLayer.forward (models/ConcatTransformer.py:171-194) with
    SelfAttResidual (transformer_modules.py:22-46) and FFResidual (:77-97)."""
    n = layer_norm(x, sd, p + ".self_attn.norm")
    qk = n + pos
    a, att = mha(qk, qk, n, sd, p + ".self_attn.sublayer", nhead, key_padding_mask=kpm)
    x = x + a
    x = x + feed_forward(layer_norm(x, sd, p + ".ff.norm"), sd, p + ".ff.sublayer")
    return x, att


def decoder_layer(y, mem, sd, p, nhead, pos, qpos, tgt_kpm, mem_kpm, tmask):
    """TransformerDecoderLayer.forward (models/ConcatTransformer.py:220-257)."""
    n = layer_norm(y, sd, p + ".tgt_self_attn.norm")
    qk = n + qpos
    a, att_s = mha(qk, qk, n, sd, p + ".tgt_self_attn.sublayer", nhead,
                   key_padding_mask=tgt_kpm, attn_mask=tmask)
    y = y + a
    n = layer_norm(y, sd, p + ".tgt_src_cross_attn.norm")
    a, att_x = mha(n + qpos, mem + pos, mem, sd, p + ".tgt_src_cross_attn.sublayer", nhead,
                   key_padding_mask=mem_kpm)
    y = y + a
    y = y + feed_forward(layer_norm(y, sd, p + ".ff.norm"), sd, p + ".ff.sublayer")
    return y, att_s, att_x


def decoder_embeddings(caps, sd, eps, padding_idx=0, p="transformer.embeddings"):
    """DecoderEmbeddings.forward (models/transformer_modules.py:113-129); the word table is an
    nn.Embedding with padding_idx=config.pad_token_id (:103-104): no gradient to that row."""
    t = caps.shape[1]
    pos_ids = torch.arange(t, dtype=torch.long).unsqueeze(0).expand(caps.shape)
    e = F.embedding(caps, sd[p + ".word_embeddings.weight"], padding_idx=padding_idx) + \
        F.embedding(pos_ids, sd[p + ".position_embeddings.weight"])
    return F.layer_norm(e, (e.shape[-1],), sd[p + ".LayerNorm.weight"],
                        sd[p + ".LayerNorm.bias"], eps)


def position_table(sd, cfg, s):
    """ConcatTransformer.positional_encoding(src) (models/ConcatTransformer.py:55) as [S, C]
    before the batch repeat: the sine table slice (models/position_encoding.py:24-35) or, for
    'learned'/'v3', LayerNorm(pos_embed(arange(S))) (position_encoding.py:50-63; its dropout is
    the identity in the parity setting, like every dropout here)."""
    if cfg.position_embedding in ("v3", "learned"):
        p = "transformer.positional_encoding"
        e = sd[p + ".pos_embed.weight"][:s]
        return F.layer_norm(e, (e.shape[-1],), sd[p + ".LayerNorm.weight"],
                            sd[p + ".LayerNorm.bias"], 1e-5)
    if s > sd["transformer.positional_encoding.pe"].shape[0]:
        raise RuntimeError(f"sequence length {s} exceeds the sine table")
    return sd["transformer.positional_encoding.pe"][:s, 0]


def transformer_forward(sd, cfg, src, m, caps, cap_mask):
    """ConcatTransformer.forward (models/ConcatTransformer.py:45-74) on already concatenated
    src [B, C, S] / mask [B, S].  Returns (hs [T, B, C], attention lists)."""
    bsz, c, s = src.shape
    nhead = cfg.nheads
    pos = position_table(sd, cfg, s).t().unsqueeze(0).repeat(bsz, 1, 1).permute(2, 0, 1)
    x = src.permute(2, 0, 1)
    tgt = decoder_embeddings(caps, sd, cfg.layer_norm_eps, cfg.pad_token_id).permute(1, 0, 2)
    qpos = sd["transformer.embeddings.position_embeddings.weight"].unsqueeze(1).repeat(1, bsz, 1)
    atts = {"enc_tc_self_att": [], "dec_exp_self_att": [], "dec_exp_tc_cross_att": []}
    for i in range(cfg.enc_layers):
        x, a = encoder_layer(x, sd, f"transformer.encoder.layers.{i}", nhead, pos, m)
        atts["enc_tc_self_att"].append(a)
    if cfg.pre_norm:           # encoder norm exists only with normalize_before (:23-24)
        x = layer_norm(x, sd, "transformer.encoder.norm")
    tmask = causal_mask(tgt.shape[0])
    y = tgt
    for i in range(cfg.dec_layers):
        y, a_s, a_x = decoder_layer(y, x, sd, f"transformer.decoder.layers.{i}", nhead, pos, qpos,
                                    cap_mask, m, tmask)
        atts["dec_exp_self_att"].append(a_s)
        atts["dec_exp_tc_cross_att"].append(a_x)
    return layer_norm(y, sd, "transformer.decoder.norm"), atts


def mlp_head(hs, sd):
    """MLP(C, 512, V, 3) (models/caption.py:161-174) on hs [T, B, C] -> logits [B, T, V]."""
    h = hs.permute(1, 0, 2)
    for i in range(3):
        h = F.linear(h, sd[f"mlp.layers.{i}.weight"], sd[f"mlp.layers.{i}.bias"])
        if i < 2:
            h = F.relu(h)
    return h


def image_tokens(sd, cfg, images, img_mask):
    """Backbone + mask interpolation + input_proj + flatten (models/caption.py:29-36)."""
    feats = resnet_body(images, sd, cfg.backbone, cfg.dilation)
    m = mask_to_features(img_mask, feats.shape[-2:])
    src = F.conv2d(feats, sd["input_proj.weight"], sd["input_proj.bias"])
    return src.flatten(2), m.flatten(1), m


def _finish(hs, atts, sd, return_attention):
    h = mlp_head(hs, sd)
    if return_attention:
        return h, {k: torch.stack(v) for k, v in atts.items()}
    return h


def caption_forward(sd, cfg, images, img_mask, caps, cap_mask, return_attention=False):
    """Caption.forward (models/caption.py:23-47) -> ConcatTransformer.forward
    (models/ConcatTransformer.py:45-74) -> MLP (models/caption.py:161-174).
    images [B,3,H,W] fp32, img_mask [B,H,W] bool, caps [B,T] int64, cap_mask [B,T] bool."""
    src, m, _ = image_tokens(sd, cfg, images, img_mask)
    hs, atts = transformer_forward(sd, cfg, src, m, caps, cap_mask)
    return _finish(hs, atts, sd, return_attention)


def caption_loc_forward(sd, cfg, images, img_mask, loc_feats, caps, cap_mask,
                        return_attention=False):
    """CaptionLoc.forward (models/caption.py:64-95): one extra memory token
    loc_proj(loc_feats) (Linear(7, C), :60) appended unmasked after the image tokens."""
    src, m, _ = image_tokens(sd, cfg, images, img_mask)
    loc = F.linear(loc_feats, sd["loc_proj.weight"], sd["loc_proj.bias"]).unsqueeze(-1)
    src = torch.concat([src, loc], 2)
    m = torch.concat([m, torch.zeros((loc_feats.shape[0], 1)).bool()], 1)
    hs, atts = transformer_forward(sd, cfg, src, m, caps, cap_mask)
    return _finish(hs, atts, sd, return_attention)


def caption_globalloc_forward(sd, cfg, t_images, t_mask, g_images, g_mask, loc_feats, caps,
                              cap_mask, return_attention=False):
    """CaptionGlobalLoc.forward (models/caption.py:113-158): target tokens, then one token per
    location feature (loc_proj = Linear(1, C) on loc_feats[..., None], :110), then the global
    context image's tokens (second backbone pass); ensure_unmasked_values (models/utils.py:
    60-89) is the identity unless a context mask is entirely True."""
    t_src, t_m, _ = image_tokens(sd, cfg, t_images, t_mask)
    loc = F.linear(loc_feats.unsqueeze(2), sd["loc_proj.weight"], sd["loc_proj.bias"])
    loc = loc.permute(0, 2, 1)
    src = torch.concat([t_src, loc], 2)
    m = torch.concat([t_m, torch.zeros((loc.shape[0], loc.shape[2])).bool()], 1)
    g_src, _, g_m = image_tokens(sd, cfg, g_images, g_mask)
    if not bool(torch.any(g_m.reshape(g_m.shape[0], -1) == False, dim=1).all()):  # noqa: E712
        raise ValueError("oracle: a fully masked context mask needs the reference's random "
                         "ensure_unmasked_values filler (not restated)")
    src = torch.concat([src, g_src], 2)
    m = torch.concat([m, g_m.flatten(1)], 1)
    hs, atts = transformer_forward(sd, cfg, src, m, caps, cap_mask)
    return _finish(hs, atts, sd, return_attention)


def caption_loss(logits, caps_out):
    """CrossEntropyLoss() (models/caption.py:210) as called at engine.py:71 — mean over B*T,
    no ignore_index (pad id 0 counts)."""
    return F.cross_entropy(logits.permute(0, 2, 1), caps_out)


def greedy(forward, batch, max_len, bos_token=1, eos_token=2):
    """eval_utils/decode.py:53-81 (with create_caption_and_mask :20-27).  ``forward(caption,
    cap_mask) -> logits [B, max_len, V]``.  Returns the caption tensor with the reference's
    exact write / early-exit semantics."""
    caption = torch.zeros((batch, max_len), dtype=torch.long)
    cap_mask = torch.ones((batch, max_len), dtype=torch.bool)
    caption[:, 0] = bos_token
    cap_mask[:, 0] = False
    finished = torch.zeros(batch, dtype=torch.bool)
    for i in range(max_len - 1):
        pred = forward(caption, cap_mask)[:, i, :]
        pid = torch.argmax(pred, axis=-1)
        finished = torch.logical_or(pid == eos_token, finished)
        if all(finished):
            return caption
        caption[:, i + 1] = pid
        cap_mask[:, i + 1] = False
    return caption


def prune_cap_ids(idx_seqs, clean=True, pad_token=0, bos_token=1, eos_token=2):
    """eval_utils/decode.py:84-101."""
    out = []
    for seq in idx_seqs:
        pr = []
        for idx in seq:
            pr.append(idx)
            if idx == eos_token:
                break
        if clean:
            pr = [i for i in pr if i not in (pad_token, bos_token, eos_token)]
        out.append(pr)
    return out


def beam_search(forward, batch, max_len, beam_size, bos_token=1, eos_token=2):
    """CPU restatement (full recompute per step) of the MI355X beam search semantics of
    retr_amd/eval_utils/decode.py IncrementalBeam / csrc/beam.hip.  The reference has NO beam
    search: this is test infrastructure for the kernels, and its only
    reference anchor is the bridge beam_size=1 == greedy (eval_utils/decode.py:53-81).
    ``forward(caption [R, T], cap_mask [R, T]) -> logits [R, T, V]`` over R = batch*beam rows
    (row b*K + k = beam k of image b).  Returns the caption [batch, T] of each image's best
    beam in greedy's format (columns after the terminating step zero)."""
    K, T = beam_size, max_len
    R = batch * K
    hist = torch.zeros((R, T), dtype=torch.long)
    hist[:, 0] = bos_token
    scores = torch.zeros(R)
    finished = torch.zeros(R, dtype=torch.bool)
    done = -1
    for i in range(T - 1):
        cm = torch.arange(T).unsqueeze(0).expand(R, T) > i
        logits = forward(hist, cm)[:, i, :].float()
        lse = torch.logsumexp(logits, -1, keepdim=True)
        vals, idx = torch.sort(logits, dim=-1, descending=True, stable=True)   # first index on ties
        lp = (vals[:, :K] - lse)
        tok = idx[:, :K]
        nh, ns, nf = hist.clone(), scores.clone(), finished.clone()
        for b in range(batch):
            cands = []                                   # (score, beam, rank-order) stable
            for k in range(K if i > 0 else 1):
                r = b * K + k
                if i > 0 and bool(finished[r]):
                    cands.append((float(scores[r]), k, int(tok[r, 0])))
                else:
                    base = float(scores[r]) if i > 0 else 0.0
                    for j in range(K):
                        cands.append((float(torch.tensor(base) + lp[r, j]), k, int(tok[r, j])))
            order = sorted(range(len(cands)), key=lambda c: (-cands[c][0], c))[:K]
            for s, c in enumerate(order):
                sc, k, t = cands[c]
                src, dst = b * K + k, b * K + s
                nh[dst] = hist[src]
                nh[dst, i + 1] = t
                ns[dst] = sc
                nf[dst] = (bool(finished[src]) if i > 0 else False) or t == eos_token
        hist, scores, finished = nh, ns, nf
        if bool(finished.all()):
            done = i
            break
    best = scores.view(batch, K).argmax(-1)
    cap = hist.view(batch, K, T)[torch.arange(batch), best].clone()
    if done >= 0:
        cap[:, done + 1:] = 0
    return cap
