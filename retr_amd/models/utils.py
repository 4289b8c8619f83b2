"""Host-side helpers with the reference's names and semantics (models/utils.py).

``NestedTensor`` (:112-133), ``nested_tensor_from_tensor_list`` (:92-109),
``generate_square_subsequent_mask`` (:50-57), ``with_pos_embed`` (:42-43), ``_get_clones``
(:46-47) and the rank helpers (:136-151).  Pure tensor plumbing — no arithmetic of the hot path.
"""
import copy
from typing import List, Optional

import torch
import torch.distributed as dist
from torch import Tensor, nn


def _max_by_axis(the_list):
    maxes = list(the_list[0])
    for sublist in the_list[1:]:
        for i, item in enumerate(sublist):
            maxes[i] = max(maxes[i], item)
    return maxes


def with_pos_embed(tensor, pos: Optional[Tensor]):
    return tensor if pos is None else tensor + pos


def _get_clones(module, n):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(n)])


def generate_square_subsequent_mask(sz):
    """Float mask: 0.0 on/below the diagonal, -inf above (models/utils.py:50-57)."""
    mask = torch.full((sz, sz), float("-inf")).triu(1)
    return mask


def ensure_unmasked_values(mask, unmasked_ratio=0.01):
    """models/utils.py:60-89: a sample whose mask is entirely True (nothing to attend to) gets a
    random filler mask with ``round(h*w*unmasked_ratio)`` positions unmasked (numpy's global
    RNG, as the reference); other samples are untouched.  Used on the global-context mask of
    CaptionGlobalLoc (models/caption.py:140)."""
    import numpy as np
    b, h, w = mask.shape
    flat = mask.reshape((b, -1))
    has_unmasked = torch.any(flat == False, dim=1)  # noqa: E712
    if False in has_unmasked:
        filler = torch.ones((h, w), dtype=bool, device=mask.device.type)
        ff = filler.flatten()
        idx = np.indices(ff.shape).flatten()
        pick = np.random.choice(idx, replace=False, size=round(idx.size * unmasked_ratio))
        ff[pick] = False
        filler = ff.reshape((h, w))
        mask[~has_unmasked] = filler
    return mask


def nested_tensor_from_tensor_list(tensor_list: List[Tensor]):
    """Zero-pad a list of [3,h,w] images to the max size; mask True on padding."""
    if tensor_list[0].ndim != 3:
        raise ValueError("not supported")
    max_size = _max_by_axis([list(img.shape) for img in tensor_list])
    b, (c, h, w) = len(tensor_list), max_size
    dev, dt = tensor_list[0].device, tensor_list[0].dtype
    tensor = torch.zeros((b, c, h, w), dtype=dt, device=dev)
    mask = torch.ones((b, h, w), dtype=torch.bool, device=dev)
    for img, pad_img, m in zip(tensor_list, tensor, mask):
        pad_img[: img.shape[0], : img.shape[1], : img.shape[2]].copy_(img)
        m[: img.shape[1], : img.shape[2]] = False
    return NestedTensor(tensor, mask)


class NestedTensor(object):
    def __init__(self, tensors, mask: Optional[Tensor]):
        self.tensors = tensors
        self.mask = mask
        self.shape = self.mask.shape

    def to(self, device):
        cast_tensor = self.tensors.to(device)
        cast_mask = self.mask.to(device) if self.mask is not None else None
        return NestedTensor(cast_tensor, cast_mask)

    def decompose(self):
        return self.tensors, self.mask

    def __repr__(self):
        return str(self.tensors)


def is_dist_avail_and_initialized():
    return dist.is_available() and dist.is_initialized()


def get_rank():
    return dist.get_rank() if is_dist_avail_and_initialized() else 0


def get_world_size():
    return dist.get_world_size() if is_dist_avail_and_initialized() else 1


def is_main_process():
    return get_rank() == 0
