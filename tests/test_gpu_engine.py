"""engine.py / eval_utils/decode.py entry points on the GPU with reference-shaped inputs:
train_one_epoch and evaluate over a loader that yields the reference's batch tuple
(ann_ids, img, mask, caps[B,129], cap_masks[B,129]) (engine.py:52-114), greedy_single and
greedy_with_att (decode.py:30-50, :131-167) and greedy_decoding (:112-128) against the
oracle's restatement of the same loops."""
import pytest
import torch

from oracle import model as orc
from retr_amd.models.utils import NestedTensor
from retr_amd.synthetic import synthetic_captions, synthetic_images, synthetic_state_dict
from tests.helpers import make_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _Set(torch.utils.data.Dataset):
    """RefCocoCaption-shaped dataset (data_utils/refcoco.py:105-188 output tuple)."""
    return_global_context = False
    return_location_features = False

    def __init__(self, cfg, n, size):
        self.img, self.mask = synthetic_images(n, size, seed=21, pad_band=True)
        self.caps, self.cm = synthetic_captions(n, cfg.max_position_embeddings, cfg.vocab_size,
                                                seed=22)
        self.annot = [(i, "img", f"caption {i}", [0, 0, 1, 1]) for i in range(n)]

    def __len__(self):
        return len(self.caps)

    def __getitem__(self, i):
        return i, self.img[i], self.mask[i], self.caps[i], self.cm[i]


def _model(cfg):
    from retr_amd.models.caption import build_model
    model, crit = build_model(cfg)
    sd = synthetic_state_dict(model, seed=42)
    model.load_state_dict(sd)
    return model.to(DEV), crit, sd


def _groups(model, cfg):
    return [{"params": [p for n, p in model.named_parameters()
                        if "backbone" not in n and p.requires_grad]},
            {"params": [p for n, p in model.named_parameters()
                        if "backbone" in n and p.requires_grad], "lr": cfg.lr_backbone}]


def test_train_one_epoch_and_evaluate():
    from retr_amd.engine import evaluate, train_one_epoch, train_step
    from retr_amd.optim import FusedAdamW
    cfg = make_config()
    ds = _Set(cfg, 6, 64)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False)
    m1, crit, sd = _model(cfg)
    m2, _, _ = _model(cfg)
    o1 = FusedAdamW(_groups(m1, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    o2 = torch.optim.AdamW(_groups(m2, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
    # evaluate at the initial weights == the oracle's mean CE over the batches
    val = evaluate(m1, crit, loader, DEV)
    ref = []
    with torch.no_grad():
        for _, img, mask, caps, cm in loader:
            lo = orc.caption_forward(sd, cfg, img, mask, caps[:, :-1], cm[:, :-1])
            ref.append(orc.caption_loss(lo, caps[:, 1:]).item())
    assert abs(val - sum(ref) / len(ref)) <= 1e-4 * abs(val)
    # one epoch == the same steps run through engine.train_step (torch AdamW + clip)
    ep = train_one_epoch(m1, crit, loader, o1, DEV, 0, cfg.clip_max_norm)
    losses = []
    m2.train()
    for _, img, mask, caps, cm in loader:
        samples = (NestedTensor(img.to(DEV), mask.to(DEV)),)
        losses.append(train_step(m2, crit, samples, caps.to(DEV), cm.to(DEV), o2,
                                 cfg.clip_max_norm).item())
    assert abs(ep - sum(losses) / len(losses)) <= 1e-4 * abs(ep)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert ((a - b).norm() / (b.norm() + 1e-30)).item() < 5e-5, n


class _Tok:
    """Tokenizer stand-in (BertTokenizer needs the HF hub): ids -> space-joined ids."""
    special = (0, 101, 102)

    def decode(self, ids, skip_special_tokens=True):
        ids = [int(i) for i in ids]
        return " ".join(str(i) for i in ids if not (skip_special_tokens and i in self.special))

    def batch_decode(self, seqs, skip_special_tokens=True):
        return [self.decode(s, skip_special_tokens) for s in seqs]


def _oracle_greedy_single(sd, cfg, img, mask, eos):
    """decode.py:30-50 restated on the oracle forward (B = 1, stop before writing EOS)."""
    T = cfg.max_position_embeddings
    cap = torch.zeros((1, T), dtype=torch.long)
    cm = torch.ones((1, T), dtype=torch.bool)
    cap[:, 0], cm[:, 0] = 101, False
    with torch.no_grad():
        for i in range(T - 1):
            pid = orc.caption_forward(sd, cfg, img, mask, cap, cm)[:, i, :].argmax(-1)
            if int(pid[0]) == eos:
                break
            cap[:, i + 1] = pid[0]
            cm[:, i + 1] = False
    return cap


def test_greedy_single_with_att_and_decoding_match_oracle():
    from retr_amd.eval_utils.decode import greedy_decoding, greedy_single, greedy_with_att
    cfg = make_config()
    model, _, sd = _model(cfg)
    img, mask = synthetic_images(1, 64, seed=31, pad_band=True)
    nt = NestedTensor(img.to(DEV), mask.to(DEV))
    tok = _Tok()
    never = _oracle_greedy_single(sd, cfg, img, mask, eos=-1)
    eos = int(never[0, 5])           # emitted mid-sequence: the early break is exercised
    ref = _oracle_greedy_single(sd, cfg, img, mask, eos)
    assert greedy_single(model, nt, tok, 101, eos, cfg.max_position_embeddings) == \
        tok.decode(ref[0])
    ids, atts = greedy_with_att(model, [nt], tok, 101, eos, cfg.max_position_embeddings)
    # with_att writes the predicted id (EOS included) before breaking (decode.py:151-158)
    j = next(c for c in range(1, never.shape[1]) if int(never[0, c]) == eos)
    assert ids.tolist() == never[0, 1:j + 1].tolist()
    assert len(atts) == j
    with torch.no_grad():
        _, att_o = orc.caption_forward(sd, cfg, img, mask, ref, ref == 0, return_attention=True)
    for k in ("enc_tc_self_att", "dec_exp_self_att", "dec_exp_tc_cross_att"):
        assert atts[0][k].shape == att_o[k].shape
    imgs, masks = synthetic_images(2, 64, seed=32, pad_band=True)
    sents = greedy_decoding([NestedTensor(imgs.to(DEV), masks.to(DEV))], model, tok,
                            max_len=cfg.max_position_embeddings, pad_token=0, bos_token=101,
                            eos_token=102)
    with torch.no_grad():
        ids_o = orc.greedy(lambda c, m: orc.caption_forward(sd, cfg, imgs, masks, c, m), 2,
                           cfg.max_position_embeddings, 101, 102)
    pruned = orc.prune_cap_ids(ids_o.tolist(), True, 0, 101, 102)
    assert sents == tok.batch_decode(pruned)
