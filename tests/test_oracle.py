"""Pin the CPU oracle (oracle/model.py) to golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import model as orc
from retr_amd.models.caption import build_model
from retr_amd.synthetic import synthetic_captions, synthetic_images, synthetic_state_dict
from tests.helpers import (F2_CASE, PARITY_CASES, VARIANT_CASES, f2_inputs, make_config,
                           variant_config, variant_inputs)

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _case(name):
    kw, size, B = PARITY_CASES[name]
    cfg = make_config(dtype="fp32", **kw)
    model, _ = build_model(cfg)        # parameter container only: gives the state_dict keys
    sd = synthetic_state_dict(model, seed=42)
    images, mask = synthetic_images(B, size, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=2)
    trainable = [n for n, p in model.named_parameters() if p.requires_grad]
    return cfg, sd, images, mask, caps, cap_mask, trainable


@pytest.mark.parametrize("name", list(PARITY_CASES))
def test_oracle_forward_backward_matches_reference(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    cfg, sd, images, mask, caps, cap_mask, trainable = _case(name)
    assert list(g["grad_names"]) == trainable          # same freeze policy as the reference
    sdo = {k: (v.clone().requires_grad_(True) if k in trainable else v) for k, v in sd.items()}
    lo = orc.caption_forward(sdo, cfg, images, mask, caps[:, :-1], cap_mask[:, :-1])
    loss = orc.caption_loss(lo, caps[:, 1:])
    loss.backward()
    lg = lo.detach()
    if "logits" in g:
        np.testing.assert_allclose(lg.numpy(), g["logits"], rtol=0, atol=2e-5)
    else:
        pos = list(g["positions"])
        np.testing.assert_allclose(lg[:, pos].numpy(), g["logits_at"], rtol=0, atol=2e-5)
    safe = g["margin"] > 1e-4
    assert (lg.argmax(-1).numpy()[safe] == g["argmax"][safe]).all()
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    norms = np.array([sdo[n].grad.norm().item() for n in trainable])
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=1e-4, atol=1e-9)
    for key in g.files:
        if key.startswith("grad/"):
            n = key[5:]
            np.testing.assert_allclose(sdo[n].grad.numpy(), g[key], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name", [n for n in PARITY_CASES if n.startswith("micro")])
def test_oracle_attention_and_greedy_match_reference(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    cfg, sd, images, mask, caps, cap_mask, _ = _case(name)
    with torch.no_grad():
        _, att = orc.caption_forward(sd, cfg, images, mask, caps[:, :-1], cap_mask[:, :-1],
                                     return_attention=True)
    for k, v in att.items():
        np.testing.assert_allclose(v.numpy(), g["att/" + k], rtol=0, atol=1e-6)
    T = cfg.max_position_embeddings
    for i, eos in enumerate(g["greedy_eos"]):
        with torch.no_grad():
            ids = orc.greedy(lambda c, m: orc.caption_forward(sd, cfg, images, mask, c, m),
                             images.shape[0], T, 101, int(eos))
        np.testing.assert_array_equal(ids.numpy(), g[f"greedy/eos{i}"])


def test_prune_cap_ids_semantics():
    seqs = [[101, 5, 6, 102, 7, 0], [101, 0, 9, 9], [101, 102, 102]]
    assert orc.prune_cap_ids(seqs, True, 0, 101, 102) == [[5, 6], [9, 9], []]
    assert orc.prune_cap_ids(seqs, False, 0, 101, 102) == [[101, 5, 6, 102], [101, 0, 9, 9],
                                                            [101, 102]]


def _variant_oracle(name, sd, cfg, images, mask, extra, caps, cap_mask, **kw):
    if cfg.use_global_features:
        (g_img, g_mask), loc = extra
        return orc.caption_globalloc_forward(sd, cfg, images, mask, g_img, g_mask, loc,
                                             caps, cap_mask, **kw)
    if cfg.use_location_features:
        return orc.caption_loc_forward(sd, cfg, images, mask, extra[0], caps, cap_mask, **kw)
    return orc.caption_forward(sd, cfg, images, mask, caps, cap_mask, **kw)


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_oracle_variants_match_reference(name):
    """CaptionLoc / CaptionGlobalLoc / learned PE / post-norm encoder."""
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    cfg = variant_config(name)
    model, _ = build_model(cfg)
    sd = synthetic_state_dict(model, seed=42)
    trainable = [n for n, p in model.named_parameters() if p.requires_grad]
    assert list(g["grad_names"]) == trainable
    images, mask, extra, caps, cap_mask = variant_inputs(name, cfg)
    sdo = {k: (v.clone().requires_grad_(True) if k in trainable else v) for k, v in sd.items()}
    lo = _variant_oracle(name, sdo, cfg, images, mask, extra, caps[:, :-1], cap_mask[:, :-1])
    loss = orc.caption_loss(lo, caps[:, 1:])
    loss.backward()
    np.testing.assert_allclose(lo.detach().numpy(), g["logits"], rtol=0, atol=2e-5)
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    norms = np.array([sdo[n].grad.norm().item() for n in trainable])
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=1e-4, atol=1e-9)


def test_oracle_f2_transformer_matches_reference():
    """F2: the 6/6 d256 transformer at S=196 (models/ConcatTransformer.py direct import)."""
    from retr_amd.models.ConcatTransformer import build_transformer
    g = np.load(os.path.join(GOLD, "f2_transformer.npz"))
    cfg = make_config(dtype="fp32", **F2_CASE)
    tr = build_transformer(cfg)
    sd = {"transformer." + k: v for k, v in synthetic_state_dict(tr, seed=43).items()}
    names = ["transformer." + n for n, _ in tr.named_parameters()]
    sdo = {k: (v.clone().requires_grad_(True) if k in names else v) for k, v in sd.items()}
    src, mask, caps, cap_mask, weight = f2_inputs(cfg)
    src.requires_grad_(True)
    hs, att = orc.transformer_forward(sdo, cfg, src, mask, caps, cap_mask)
    (hs * weight).sum().backward()
    np.testing.assert_allclose(hs.detach().numpy(), g["hs"], rtol=0, atol=3e-5)
    np.testing.assert_allclose(src.grad.numpy(), g["src_grad"], rtol=0, atol=1e-4)
    for k, v in att.items():
        np.testing.assert_allclose(torch.stack(v).detach()[:, :, ::7].numpy(), g["att/" + k],
                                   rtol=0, atol=1e-6)
    assert [n[len("transformer."):] for n in names] == list(g["grad_names"])
    norms = np.array([sdo[n].grad.norm().item() for n in names])
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("name", [n for n in PARITY_CASES if n.startswith("micro")])
def test_oracle_beam1_is_reference_greedy(name):
    """The beam-search restatement (no reference implementation exists) is anchored to the
    reference through beam_size=1 == eval_utils/decode.py greedy, on the reference's own ids."""
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    cfg, sd, images, mask, caps, cap_mask, _ = _case(name)
    T = cfg.max_position_embeddings
    for i, eos in enumerate(g["greedy_eos"]):
        with torch.no_grad():
            ids = orc.beam_search(lambda c, m: orc.caption_forward(sd, cfg, images, mask, c, m),
                                  images.shape[0], T, 1, 101, int(eos))
        np.testing.assert_array_equal(ids.numpy(), g[f"greedy/eos{i}"])
