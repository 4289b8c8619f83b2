"""Non-default reference surfaces on the GPU against the reference's own outputs
(tests/golden/*.npz from tests/golden/make_golden.py), fp32 parity mode:

* CaptionLoc (models/caption.py:50-95) incl. the reference's Linear(7)-vs-5-features error;
* CaptionGlobalLoc (models/caption.py:98-158), incl. a fully masked context image;
* learned position embeddings ('learned', models/position_encoding.py:38-63);
* pre_norm=False (no encoder final LayerNorm, models/ConcatTransformer.py:24);
* F2: the 6/6 d256 nhead-8 transformer at S=196, T=128 through
  ConcatTransformer.forward's reference signature.
"""
import os

import numpy as np
import pytest
import torch

from retr_amd.models.caption import build_model
from retr_amd.models.utils import NestedTensor
from retr_amd.synthetic import synthetic_images, synthetic_state_dict
from tests.helpers import F2_CASE, VARIANT_CASES, f2_inputs, make_config, variant_config, \
    variant_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _variant_model(name, dtype="fp32"):
    cfg = variant_config(name, dtype)
    model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=42))
    return cfg, model.to(DEV), crit


def _args(cfg, images, mask, extra):
    args = [NestedTensor(images.to(DEV), mask.to(DEV))]
    for e in extra:
        args.append(NestedTensor(e[0].to(DEV), e[1].to(DEV)) if isinstance(e, tuple)
                    else e.to(DEV))
    return args


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_variant_matches_reference_golden(name):
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    cfg, model, crit = _variant_model(name)
    pe = model.transformer.positional_encoding
    if hasattr(pe, "dropout"):
        pe.dropout.p = 0.0          # as the generator did (reference fixes it at 0.1)
    images, mask, extra, caps, cap_mask = variant_inputs(name, cfg)
    model.train()
    out = model(*_args(cfg, images, mask, extra), caps[:, :-1].to(DEV),
                cap_mask[:, :-1].to(DEV))
    loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
    loss.backward()
    assert _rel(out.detach().float(), g["logits"]) < 1e-3
    assert abs(loss.item() - float(g["loss"])) <= 1e-3 * abs(float(g["loss"]))
    params = dict(model.named_parameters())
    assert list(g["grad_names"]) == [n for n, p in params.items() if p.requires_grad]
    norms = np.array([params[n].grad.norm().item() for n in g["grad_names"]])
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=2e-3, atol=1e-7)


def test_caption_loc_five_features_raise_like_reference():
    """The dataset's position features have 5 entries (data_utils/utils.py:200-237) while
    CaptionLoc.loc_proj is Linear(7, C): the reference fails in F.linear; so does this."""
    cfg, model, _ = _variant_model("micro_loc")
    images, mask, extra, caps, cap_mask = variant_inputs("micro_loc", cfg)
    with pytest.raises(RuntimeError, match="mat1 and mat2 shapes cannot be multiplied"):
        model(NestedTensor(images.to(DEV), mask.to(DEV)), torch.rand(2, 5, device=DEV),
              caps[:, :-1].to(DEV), cap_mask[:, :-1].to(DEV))


def test_global_loc_fully_masked_context_runs():
    """ensure_unmasked_values (models/utils.py:60-89) un-masks a random 1% of a fully padded
    context mask so no attention row is all -inf."""
    cfg, model, crit = _variant_model("micro_globalloc", "bf16")
    images, mask, extra, caps, cap_mask = variant_inputs("micro_globalloc", cfg)
    g_img, g_mask = synthetic_images(2, 64, seed=9)
    g_mask[1] = True
    extra[0] = (g_img, g_mask)
    np.random.seed(0)
    out = model(*_args(cfg, images, mask, extra), caps[:, :-1].to(DEV),
                cap_mask[:, :-1].to(DEV))
    loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
    loss.backward()
    assert torch.isfinite(loss) and torch.isfinite(out.float()).all()


def test_learned_pe_training_dropout_runs_bf16():
    """Learned PE in training mode keeps its fixed p=0.1 dropout (a fresh mask per sample)."""
    cfg, model, crit = _variant_model("micro_learned_pe", "bf16")
    cfg.dropout = 0.1
    images, mask, extra, caps, cap_mask = variant_inputs("micro_learned_pe", cfg)
    model.train()
    out = model(NestedTensor(images.to(DEV), mask.to(DEV)), caps[:, :-1].to(DEV),
                cap_mask[:, :-1].to(DEV))
    loss = crit(out.permute(0, 2, 1), caps[:, 1:].to(DEV))
    loss.backward()
    pw = model.transformer.positional_encoding.pos_embed.weight.grad
    assert torch.isfinite(pw).all()
    S = 4    # R18 at 64x64: 2x2 feature grid
    assert pw[:S].abs().sum() > 0 and pw[S:].abs().sum() == 0


def test_f2_transformer_matches_reference_golden():
    """SURVEY §8(c) F2 through ConcatTransformer.forward(src_t, mask_t, src_c, mask_c, tgt,
    tgt_mask) -> (hs [T, B, C], atts), fp32 parity mode, against the reference module's own
    output, attention maps and gradients."""
    from retr_amd.models.ConcatTransformer import build_transformer
    g = np.load(os.path.join(GOLD, "f2_transformer.npz"))
    cfg = make_config(dtype="fp32", **F2_CASE)
    tr = build_transformer(cfg)
    tr.load_state_dict(synthetic_state_dict(tr, seed=43))
    tr.to(DEV).train()
    tr.cdtype = torch.float32
    src, mask, caps, cap_mask, weight = f2_inputs(cfg)
    src = src.to(DEV).requires_grad_(True)
    hs, atts = tr(src, mask.to(DEV), None, None, caps.to(DEV), cap_mask.to(DEV))
    (hs.float() * weight.to(DEV)).sum().backward()
    assert _rel(hs.detach().float(), g["hs"]) < 1e-3
    assert _rel(src.grad, g["src_grad"]) < 2e-3
    for k, v in atts.items():
        assert _rel(v[:, :, ::7].float(), g["att/" + k]) < 1e-3, k
    params = dict(tr.named_parameters())
    norms = np.array([params[n].grad.norm().item() for n in g["grad_names"]])
    np.testing.assert_allclose(norms, g["grad_norms"], rtol=2e-3, atol=1e-7)
