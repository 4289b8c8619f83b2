"""Deterministic synthetic weights and RefCOCO-shaped inputs (no network, no datasets).

Weights: one numpy PCG64 stream per ``state_dict`` key (seeded by (seed, crc32(key))), so the
same key gets the same values on any machine and independent of model construction order.
Scales are calibrated analytically so activations stay O(1) through deep ResNets (SURVEY.md
§0.5): He-normal convs, FrozenBN with unit-ish statistics and the last BN of every residual
branch scaled by 0.2.

Inputs follow SURVEY.md §8d: images ~ N(0,1) (post-Normalize statistics); captions
[B, T+1] = BOS, L~U{3..20} word ids, EOS, pad 0; cap_mask = (caps == 0).
"""
import zlib

import numpy as np
import torch


def _rng(seed, key):
    return np.random.default_rng([int(seed), zlib.crc32(key.encode())])


def _is_bn(key):
    return (".bn" in key or "downsample.1." in key) and key.startswith("backbone.")


def _last_bn_of_branch(key, kind):
    return (kind == "bottleneck" and ".bn3." in key) or (kind == "basic" and ".bn2." in key)


def synthetic_state_dict(model, seed=42):
    """Synthetic values for every entry of ``model.state_dict()`` (fp32, CPU), except the fixed
    sine table ``transformer.positional_encoding.pe`` which keeps its computed value."""
    sd = model.state_dict()
    kind = "bottleneck" if any(".conv3." in k for k in sd) else "basic"
    out = {}
    for key, t in sd.items():
        shape = tuple(t.shape)
        r = _rng(seed, key)
        if key.endswith("positional_encoding.pe"):
            out[key] = t.detach().clone().float().cpu()
            continue
        if _is_bn(key):
            leaf = key.rsplit(".", 1)[1]
            if leaf == "weight":
                v = r.uniform(0.8, 1.2, shape)
                if _last_bn_of_branch(key, kind):
                    v = v * 0.2
            elif leaf == "bias":
                v = r.normal(0.0, 0.05, shape)
            elif leaf == "running_mean":
                v = r.normal(0.0, 0.05, shape)
            elif leaf == "running_var":
                v = r.uniform(0.8, 1.2, shape)
            else:
                v = np.zeros(shape)
        elif len(shape) == 4:                          # conv weights (OIHW)
            fan_in = shape[1] * shape[2] * shape[3]
            v = r.normal(0.0, np.sqrt(2.0 / fan_in), shape)
            if key.startswith("input_proj"):
                v = r.normal(0.0, np.sqrt(1.0 / fan_in), shape)
        elif "norm" in key.lower():                    # LayerNorm affine
            v = 1.0 + r.normal(0.0, 0.1, shape) if key.endswith("weight") else \
                r.normal(0.0, 0.05, shape)
        elif len(shape) == 2:                          # linear / in_proj / embeddings: xavier
            a = np.sqrt(6.0 / (shape[0] + shape[1]))
            v = r.uniform(-a, a, shape)
        elif len(shape) == 1:                          # biases
            v = r.normal(0.0, 0.02, shape)
        else:
            v = t.detach().cpu().numpy()
        out[key] = torch.from_numpy(np.asarray(v, dtype=np.float32).reshape(shape))
    return out


def synthetic_images(batch, size, seed=0, pad_band=False):
    """images [B, 3, H, H] fp32 ~ N(0,1); mask [B, H, H] bool.  ``pad_band`` marks columns
    [0, H/8) and [7H/8, H) as padding (pad_mask_to_max, data_utils/utils.py:242-255)."""
    r = np.random.default_rng([int(seed), 1])
    img = torch.from_numpy(r.standard_normal((batch, 3, size, size), dtype=np.float32))
    mask = torch.zeros(batch, size, size, dtype=torch.bool)
    if pad_band:
        q = size // 8
        mask[:, :, :q] = True
        mask[:, :, size - q:] = True
        img = img.masked_fill(mask[:, None], 0.0)
    return img, mask


def synthetic_captions(batch, max_len, vocab_size, seed=0, bos=101, eos=102, pad=0):
    """caps [B, max_len+1] int64 and cap_mask (caps == pad) (data_utils/refcoco.py:95-124)."""
    r = np.random.default_rng([int(seed), 2])
    caps = np.zeros((batch, max_len + 1), dtype=np.int64)
    lo = min(1000, vocab_size // 2)
    for b in range(batch):
        n = int(r.integers(3, 21))
        n = min(n, max_len - 1)
        caps[b, 0] = bos
        caps[b, 1:1 + n] = r.integers(lo, vocab_size, n)
        caps[b, 1 + n] = eos
    caps = torch.from_numpy(caps)
    return caps, caps == pad


class SyntheticRefDataset(torch.utils.data.Dataset):
    """RefCocoCaption-shaped dataset (the output tuple of data_utils/refcoco.py:105-188:
    ann_id, image [3, H, H], mask [H, H], caps [T+1], cap_mask [T+1]) on synthetic data, for
    the data-parallel launcher and its tests (RefCOCO itself is not fetched here)."""
    return_global_context = False
    return_location_features = False

    def __init__(self, config, n, size, seed=0):
        self.img, self.mask = synthetic_images(n, size, seed=31 + seed, pad_band=True)
        self.caps, self.cap_mask = synthetic_captions(n, config.max_position_embeddings,
                                                      config.vocab_size, seed=32 + seed)
        self.annot = [(i, "img", f"caption {i}", [0, 0, 1, 1]) for i in range(n)]

    def __len__(self):
        return len(self.caps)

    def __getitem__(self, i):
        return i, self.img[i], self.mask[i], self.caps[i], self.cap_mask[i]
