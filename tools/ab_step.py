"""A/B timing of the graphed cfg2 training step under code-path variants, in ONE process with
interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Each variant is a dict of switches
applied before its own capture; prints per-variant median / min ms per step.

    python tools/ab_step.py --variants base,side_all --rounds 5 --steps 10
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from retr_amd import ops, resnet  # noqa: E402
from retr_amd._lib import load  # noqa: E402
from retr_amd.engine import GraphedTrainStep  # noqa: E402
from retr_amd.models.utils import NestedTensor  # noqa: E402
from retr_amd.synthetic import synthetic_captions, synthetic_images  # noqa: E402

VARIANTS = {
    "base": {},
    "side_bb": {("OVERLAP", "backbone"): True},
    "side_tr": {("OVERLAP", "transformer"): True},
    "side_all": {("OVERLAP", "backbone"): True, ("OVERLAP", "transformer"): True},
    "nofuse_ln": {("ATTR", "FUSE_LN_BWD"): False},
    "no_lnparams": {("ATTR", "FUSE_LN_PARAMS"): False},
    "no_dmask": {("ATTR", "ATTN_DMASK"): False},
    "split_off": {("TUNE", 10): 1},
    "split_all": {("TUNE", 10): 2},
    "split_dq_all": {("TUNE", 10): 2},
    "no_dmask_split_off": {("ATTR", "ATTN_DMASK"): False, ("TUNE", 10): 1},
    "no_stem_pool": {("ENV", "RETR_STEM_POOL"): "0"},
    "lin_small": {("TUNE", 13): 2},
    "fsplit_off": {("TUNE", 12): 1},
    "shortk_off": {("TUNE", 14): 1},
    "grp_s1": {("TUNE", 1): 1},
    "wgrp_s1": {("TUNE", 3): 1},
    "cwg_s1": {("TUNE", 9): 3},
    "adamw_nt": {("TUNE", 15): 1},
    "adamw_plain": {("TUNE", 15): 2},
    "adamw_u2": {("TUNE", 15): 3},
    "lin_k256": {("TUNE", 33): 2},
    "lin_k256_loop": {("TUNE", 33): 1},
    "gemm_nt": {("TUNE", 7): 1},
    "ce_unfused": {("ATTR", "FUSED_CE"): False},
    "wgrad_b64": {("TUNE", 16): 1},
    "grp_s4": {("TUNE", 1): 4},
    "wgrp_s4": {("TUNE", 3): 4},
    "wkc256": {("TUNE", 4): 256},
    "wkc1024": {("TUNE", 4): 1024},
    "wtile128": {("TUNE", 2): 128},
    "wthr50k": {("TUNE", 2): 50000},
    "wthr100k": {("TUNE", 2): 100000},
    "wthr120k": {("TUNE", 2): 120000},
    "wthr400k": {("TUNE", 2): 400000},
    "wgrad_fused": {("TUNE", 17): 1},
    "ffn_fused": {("ATTR", "FUSE_FFN"): True},
    "wkc2048": {("TUNE", 4): 2048},
    "wkc3200": {("TUNE", 4): 3200},
    "wdefer_off": {("ATTR", "WGRAD_DEFER"): False},
    "wb64": {("TUNE", 2): 64},
    "wb128": {("TUNE", 2): 128},
    "wside_on": {("ATTR", "WGRAD_SIDE"): True},
    "cwg_off": {("RESNET", "CONV_WGRAD_GROUP"): False},
    "skf": {("TUNE", 18): 1},
    "wbc16": {("TUNE", 19): 16},
    "wbc64": {("TUNE", 19): 64},
    "cwc16": {("TUNE", 20): 16},
    "cwc64": {("TUNE", 20): 64},
    "c16": {("TUNE", 19): 16, ("TUNE", 20): 16},
    "c3_off": {("TUNE", 21): 1},
    "panel_on": {("TUNE", 23): 1},
    "pg4": {("TUNE", 23): 1, ("TUNE", 24): 4},
    "pg16": {("TUNE", 23): 1, ("TUNE", 24): 16},
    "pconv": {("TUNE", 23): 1, ("TUNE", 25): 1},
    "kb_on": {("TUNE", 26): 1},
    "lnn_off": {("ATTR", "FUSE_LN_NEXT"): False},
    "hd_off": {("ATTR", "HEAD_WGRAD_DEFER"): False},
    "pos_on": {("ATTR", "POS_DEFER"): True},
    "pos_off": {("ATTR", "POS_DEFER"): False},
    "up2k": {("TUNE", 28): 2048},
    "up8k": {("TUNE", 28): 8192},
    # round 6: round 5's conv weight-gradient unpack (block per 64 chunks) vs the row kernel
    "unpack_old": {("TUNE", 28): -1},
    # round 6: the first blocks' downsample data gradient out of place (+ phase fill)
    "ds_fill": {("RESNET", "DS_DGRAD_INPLACE"): False},
    "lnslab_off": {("ATTR", "LN_BWD_SLABS"): False},
    # grouped projection tiles (RETR_TUNE_GROUP_TILE / _STAGES) re-check
    "grp_t128": {("TUNE", 0): 128},
    "grp_t128s1": {("TUNE", 0): 128, ("TUNE", 1): 1},
    "grp_t128s3": {("TUNE", 0): 128, ("TUNE", 1): 3},
    "cw_w4": {("TUNE", 29): 1},
    "cw_w8": {("TUNE", 29): 2},
    "cw_256": {("TUNE", 29): 3},
}


def apply(v):
    ops.OVERLAP.update({"backbone": False, "transformer": False})
    ops.FUSE_LN_BWD = True
    ops.FUSE_LN_PARAMS = True
    ops.ATTN_DMASK = True
    ops.FUSED_CE = True
    ops.FUSE_FFN = False
    ops.WGRAD_DEFER = True
    ops.WGRAD_SIDE = False
    ops.FUSE_LN_NEXT = True
    ops.HEAD_WGRAD_DEFER = True
    ops.POS_DEFER = True
    ops.LN_BWD_SLABS = True
    resnet.CONV_WGRAD_GROUP = True
    resnet.DS_DGRAD_INPLACE = True
    load().retr_tune(10, 0)
    load().retr_tune(12, 0)
    load().retr_tune(13, 0)
    load().retr_tune(14, 0)
    for k in (0, 1, 2, 3, 4, 7, 9, 15, 16, 17, 18, 19, 20, 21, 23, 24, 25, 26, 27, 28, 29, 32, 33):
        load().retr_tune(k, 0)
    ops._SPLITS.clear()                        # split-K counts are cached per shape
    os.environ["RETR_STEM_POOL"] = "1"
    for (table, key), val in VARIANTS[v].items():
        if table == "ENV":                     # read when the model is built
            os.environ[key] = val
        elif table == "ATTR":
            setattr(ops, key, val)
        elif table == "RESNET":
            setattr(resnet, key, val)
        elif table == "TUNE":
            load().retr_tune(key, val)
        else:
            getattr(ops, table)[key] = val


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base,side_all")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = bench.cfg2()
    names = args.variants.split(",")
    runs = {}
    img, mask = synthetic_images(16, 640, seed=1000)
    caps, cm = synthetic_captions(16, 128, cfg.vocab_size, seed=2000)
    samples = (NestedTensor(img.to(dev), mask.to(dev)),)
    caps, cm = caps.to(dev), cm.to(dev)
    for v in names:
        apply(v)
        model, crit = bench.build(cfg, dev)
        model.train()
        opt = bench.make_optimizer(model, cfg, fused=True)
        g = GraphedTrainStep(model, crit, opt, cfg.clip_max_norm)
        g(samples, caps, cm)
        torch.cuda.synchronize()
        runs[v] = g
    res = {v: [] for v in names}
    for _ in range(args.rounds):
        for v in names:
            g = runs[v]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                g(samples, caps, cm)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / args.steps * 1e3)
    for v in names:
        print(f"{v:14s} median {statistics.median(res[v]):7.3f} ms  min {min(res[v]):7.3f} ms  "
              f"rounds {[round(x, 3) for x in res[v]]}")


if __name__ == "__main__":
    main()
