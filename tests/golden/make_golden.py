"""Generate the golden vectors that pin the CPU oracle (run in the BUILD container only).

It imports the reference itself from /root/reference (read-only) and runs its own code:
``models.caption.build_model`` -> ``Caption.forward`` -> ``CrossEntropyLoss`` -> backward,
``return_attention=True`` maps, and ``eval_utils.decode.greedy``.  torchvision (a third-party
dependency of the reference, absent from this image, version unpinned) is provided by the
restatement in ``oracle/tv_resnet.py``; everything else is the reference's code.

Inputs are fully deterministic (retr_amd.synthetic: numpy PCG64 per state_dict key; images /
captions from fixed seeds), so the fixtures store only outputs and the tests regenerate inputs.

    python tests/golden/make_golden.py [case ...]   # writes tests/golden/*.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

from oracle.tv_resnet import install_torchvision_standin  # noqa: E402
from retr_amd.synthetic import (synthetic_captions, synthetic_images,  # noqa: E402
                                synthetic_state_dict)
from tests.helpers import (F2_CASE, PARITY_CASES, VARIANT_CASES, f2_inputs,  # noqa: E402
                           make_config, variant_config, variant_inputs)

SMALL_GRADS = ("input_proj.bias", "transformer.decoder.norm.weight", "mlp.layers.2.bias",
               "transformer.embeddings.position_embeddings.weight",
               "transformer.embeddings.LayerNorm.weight",
               "transformer.encoder.layers.0.self_attn.sublayer.in_proj_bias",
               "transformer.decoder.layers.0.tgt_src_cross_attn.sublayer.out_proj.bias",
               "backbone.body.layer2.0.conv1.weight")
CFG1_POSITIONS = [0, 1, 2, 5, 17, 63, 127]


def ref_modules():
    import transformers  # noqa: F401  (imported before the stand-in: it probes torchvision)
    install_torchvision_standin()
    sys.path.insert(0, REF)
    import importlib
    caption = importlib.import_module("models.caption")
    utils = importlib.import_module("models.utils")
    decode = importlib.import_module("eval_utils.decode")
    return caption, utils, decode


def make_case(name, caption, utils, decode):
    kw, size, B = PARITY_CASES[name]
    cfg = make_config(dtype="fp32", **kw)
    torch.manual_seed(0)
    model, criterion = caption.build_model(cfg)
    sd = synthetic_state_dict(model, seed=42)
    model.load_state_dict(sd)
    images, mask = synthetic_images(B, size, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=2)
    out = {}
    model.train()   # dropout=0 -> deterministic; grads follow the reference freeze policy
    samples = utils.NestedTensor(images, mask)
    logits = model(samples, caps[:, :-1], cap_mask[:, :-1])
    loss = criterion(logits.permute(0, 2, 1), caps[:, 1:])
    loss.backward()
    out["loss"] = np.float64(loss.item())
    lg = logits.detach()
    if lg.numel() <= 2_000_000:
        out["logits"] = lg.numpy()
    else:
        out["positions"] = np.array(CFG1_POSITIONS)
        out["logits_at"] = lg[:, CFG1_POSITIONS].numpy()
    top2 = lg.topk(2, dim=-1).values
    out["argmax"] = lg.argmax(-1).numpy()
    out["margin"] = (top2[..., 0] - top2[..., 1]).numpy()
    names, norms = [], []
    for n, p in model.named_parameters():
        if p.requires_grad:
            names.append(n)
            norms.append(p.grad.norm().item())
            if n in SMALL_GRADS:
                out["grad/" + n] = p.grad.numpy()
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array(norms)
    if name.startswith("micro"):
        model.eval()
        with torch.no_grad():
            _, att = model(samples, caps[:, :-1], cap_mask[:, :-1], return_attention=True)
        for k, v in att.items():
            out["att/" + k] = v.numpy()
        T = cfg.max_position_embeddings
        with torch.no_grad():
            never = decode.greedy([samples], model, max_len=T, device="cpu", bos_token=101,
                                  eos_token=-1)
            eos_list = [-1, int(never[0, 6]), int(never[0, 1])]
            for i, eos in enumerate(eos_list):
                ids = decode.greedy([samples], model, max_len=T, device="cpu", bos_token=101,
                                    eos_token=eos)
                out[f"greedy/eos{i}"] = ids.numpy()
        out["greedy_eos"] = np.array(eos_list)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.0f} kB) loss={out['loss']:.6f}")


def _grads(model, out):
    names, norms = [], []
    for n, p in model.named_parameters():
        if p.requires_grad and p.grad is not None:
            names.append(n)
            norms.append(p.grad.norm().item())
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array(norms)


def make_variant(name, caption, utils):
    """Non-default reference surfaces (pre_norm=False): CaptionLoc,
    CaptionGlobalLoc, learned position embeddings, post-norm encoder (no final LayerNorm)."""
    cfg = variant_config(name)
    torch.manual_seed(0)
    model, criterion = caption.build_model(cfg)
    sd = synthetic_state_dict(model, seed=42)
    model.load_state_dict(sd)
    pe = model.transformer.positional_encoding
    if hasattr(pe, "dropout"):
        pe.dropout.p = 0.0      # the learned PE's own dropout is fixed at 0.1 in the reference
    images, mask, extra, caps, cap_mask = variant_inputs(name, cfg)
    args = [utils.NestedTensor(images, mask)]
    for e in extra:
        args.append(utils.NestedTensor(*e) if isinstance(e, tuple) else e)
    model.train()
    logits = model(*args, caps[:, :-1], cap_mask[:, :-1])
    loss = criterion(logits.permute(0, 2, 1), caps[:, 1:])
    loss.backward()
    out = {"loss": np.float64(loss.item()), "logits": logits.detach().numpy()}
    _grads(model, out)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.0f} kB) loss={out['loss']:.6f}")


def make_f2(ct_module):
    """the transformer half at real depth (6/6, d256, nhead 8, S=196, T=128)
    imported directly from models/ConcatTransformer.py (no torchvision shim involved)."""
    kw = F2_CASE
    cfg = make_config(dtype="fp32", **kw)
    torch.manual_seed(0)
    tr = ct_module.build_transformer(cfg)
    sd = synthetic_state_dict(tr, seed=43)
    tr.load_state_dict(sd)
    tr.train()
    src, mask, caps, cap_mask, weight = f2_inputs(cfg)
    src.requires_grad_(True)
    hs, atts = tr(src, mask, None, None, caps, cap_mask)
    (hs * weight).sum().backward()
    out = {"hs": hs.detach().numpy(), "src_grad": src.grad.numpy()}
    for k, v in atts.items():
        out["att/" + k] = v.detach()[:, :, ::7].numpy()       # every 7th query row
    _grads(tr, out)
    path = os.path.join(HERE, "f2_transformer.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.0f} kB)")


def main():
    caption, utils, decode = ref_modules()
    import importlib
    ct = importlib.import_module("models.ConcatTransformer")
    which = sys.argv[1:] or (list(PARITY_CASES) + list(VARIANT_CASES) + ["f2"])
    for name in which:
        if name in PARITY_CASES:
            make_case(name, caption, utils, decode)
        elif name in VARIANT_CASES:
            make_variant(name, caption, utils)
        elif name == "f2":
            make_f2(ct)


if __name__ == "__main__":
    main()
