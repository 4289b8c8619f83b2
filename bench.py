"""RE⫶TR hot-path benchmark on MI355X (BASELINE.json metric).

Step = one reference training step (engine.py:70-83): Caption forward, CrossEntropy, backward,
RCCL gradient all-reduce (N>1), clip_grad_norm_(0.1), AdamW — on BASELINE config 2
(ResNet-50 + 6/6 encoder/decoder, d_model 256, 640x640 RefCOCO-shaped synthetic batch of 16
per GPU, bf16 operands / fp32 master weights, dropout 0.1).  Also reported: greedy-decode
refs/sec on config 5 (ResNet-50 dilation=True 224x224, batch 64, 127 steps) and the CPU
oracle timed on this host's cores.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...    (one process per GPU, RCCL)
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from retr_amd.configuration import Config  # noqa: E402
from retr_amd.models.caption import build_model  # noqa: E402
from retr_amd.models.utils import NestedTensor  # noqa: E402
from retr_amd.synthetic import (synthetic_captions, synthetic_images,  # noqa: E402
                                synthetic_state_dict)
from retr_amd import probe as probe_mod  # noqa: E402

METRIC = "RefCOCO images/sec (train fwd+bwd) at 1/2/4/8 GPUs; greedy-decode refs/sec"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def cfg2(dtype="bf16"):
    c = Config()
    c.backbone, c.dilation, c.hidden_dim = "ResNet50", False, 256
    c.enc_layers = c.dec_layers = 6
    c.nheads, c.dim_feedforward, c.dropout = 8, 2048, 0.1
    c.lr_backbone, c.lr, c.weight_decay = 1e-5, 1e-4, 1e-4
    c.dtype = dtype
    return c


def cfg5(dtype="bf16"):
    c = cfg2(dtype)
    c.dilation = True
    return c


def build(cfg, device, seed=42):
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):    # build_model's prints (caption.py:204,211)
        model, crit = build_model(cfg)
    model.load_state_dict(synthetic_state_dict(model, seed=seed))
    return model.to(device), crit


def make_optimizer(model, cfg, capturable=False, fused=False):
    """main.py:30-39: two param groups (backbone at lr_backbone), AdamW — torch's, or with
    ``fused`` the MI355X FusedAdamW (clip + AdamW in two kernels over flat arenas)."""
    groups = [{"params": [p for n, p in model.named_parameters()
                          if "backbone" not in n and p.requires_grad]},
              {"params": [p for n, p in model.named_parameters()
                          if "backbone" in n and p.requires_grad], "lr": cfg.lr_backbone}]
    if fused:
        from retr_amd.optim import FusedAdamW
        return FusedAdamW(groups, lr=cfg.lr, weight_decay=cfg.weight_decay)
    return torch.optim.AdamW(groups, lr=cfg.lr, weight_decay=cfg.weight_decay,
                             capturable=capturable)


def train_bench(args, rank, world, device):
    from retr_amd.engine import GraphedTrainStep, train_step
    cfg = cfg2()
    model, crit = build(cfg, device)
    graphed = not args.eager
    sync = None
    if world > 1:
        from retr_amd.ddp import broadcast_parameters
        broadcast_parameters(model)
    opt = make_optimizer(model, cfg, capturable=graphed, fused=not args.torch_adamw)
    if world > 1:
        # zero-copy buckets on FusedAdamW's gradient arena; a graphed step runs them between
        # its forward/backward graph and its optimizer graph
        from retr_amd.ddp import GradSync
        sync = GradSync([p for p in model.parameters() if p.requires_grad],
                        bucket_mb=cfg.grad_bucket_mb, optimizer=opt)
    B, H = args.batch, args.size
    img, mask = synthetic_images(B, H, seed=1000 + rank)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size,
                                        seed=2000 + rank)
    samples = (NestedTensor(img.to(device), mask.to(device)),)
    caps, cap_mask = caps.to(device), cap_mask.to(device)
    model.train()

    def eager_step():
        return train_step(model, crit, samples, caps, cap_mask, opt, cfg.clip_max_norm, sync)

    graph_step = GraphedTrainStep(model, crit, opt, cfg.clip_max_norm, sync) if graphed else None

    def step():
        if graph_step is not None:
            return graph_step(samples, caps, cap_mask)
        return eager_step()

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item(), "non-finite loss in warmup"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    loss_v = float(loss.item())
    # per-kernel HIP-event timing needs host-side launches: after the timed region, re-run the
    # identical step eagerly (same weights / inputs / stream) with the probe on
    pr = probe_mod.Probe(detail=bool(args.probe_detail))
    with pr:
        for _ in range(args.probe_steps):
            eager_step()
    torch.cuda.synchronize()
    fam = pr.summary()
    if args.probe_detail and rank == 0:
        nst = max(1, args.probe_steps)
        with open(args.probe_detail, "w") as f:
            for k, v in sorted(fam.items(), key=lambda kv: -kv[1]["ms_total"]):
                f.write(f"{v['ms_total'] / nst:8.3f} ms/step {v['launches'] // nst:4d}x "
                        f"{v['ms_avg'] * 1e3:8.1f} us {v['tflops']:7.1f} TF/s  {k}\n")
        fam = {}
        for k, v in pr.summary().items():
            d = fam.setdefault(k.split(" | ")[0], {"launches": 0, "ms_total": 0.0,
                                                   "flops": 0.0})
            for f in ("launches", "ms_total", "flops"):
                d[f] += v[f]
        for d in fam.values():
            d["ms_avg"] = d["ms_total"] / max(1, d["launches"])
            d["tflops"] = d["flops"] / (d["ms_total"] * 1e-3) / 1e12 if d["ms_total"] else 0.0
    return dt, loss_v, fam, max(1, args.probe_steps)


def decode_bench(args, rank, world, device):
    """cfg5 decode: greedy (the reference's algorithm, KV-cache incremental form) and beam
    search (beam 5; new capability) refs/sec over one batch, hipGraph-replayed steps."""
    from retr_amd.eval_utils.decode import IncrementalBeam, greedy
    cfg = cfg5()
    model, _ = build(cfg, device)
    model.eval()
    B = args.decode_batch
    img, mask = synthetic_images(B, 224, seed=3000 + rank)
    samples = [NestedTensor(img.to(device), mask.to(device))]
    T = cfg.max_position_embeddings
    out = {}
    runs = [("greedy", lambda: greedy(samples, model, max_len=T, bos_token=101, eos_token=102))]
    if args.beam > 1:
        beam = IncrementalBeam(model, args.beam)
        runs.append((f"beam{args.beam}", lambda: beam(samples, T, 101, 102)))
    for name, fn in runs:
        ids = fn()                                  # warm-up (captures the step graphs)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        ids = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = t.item()
        out[name] = (dt, int((ids != 0).sum(1).max().item()))
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args):
    """CPU oracle (oracle/model.py: fp32 eager torch in the reference's op order, pinned to the
    reference by tests/golden) on this host: fwd + CE + backward of config 2 on a bounded
    sample (batch 2, 640x640), timed steps until ``--cpu-seconds`` have elapsed."""
    from oracle import model as orc
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    torch.set_num_threads(cores)
    cfg = cfg2("fp32")
    cfg.dropout = 0.0
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):
        model, _ = build_model(cfg)
    sd = synthetic_state_dict(model, seed=42)
    trainable = {n for n, p in model.named_parameters() if p.requires_grad}
    sd = {k: (v.requires_grad_(True) if k in trainable else v) for k, v in sd.items()}
    B = 2
    img, mask = synthetic_images(B, args.size, seed=1)
    caps, cap_mask = synthetic_captions(B, cfg.max_position_embeddings, cfg.vocab_size, seed=2)

    def step():
        for v in sd.values():
            v.grad = None
        lo = orc.caption_forward(sd, cfg, img, mask, caps[:, :-1], cap_mask[:, :-1])
        orc.caption_loss(lo, caps[:, 1:]).backward()

    step()
    n = 0
    t0 = time.perf_counter()
    while True:
        step()
        n += 1
        dt = time.perf_counter() - t0
        if (n >= 2 and dt >= args.cpu_seconds) or n >= 50:
            break
    return {"value": round(B * n / dt, 4), "unit": "images/s", "cores": cores, "kind": "port",
            "cpu": _cpu_model(), "seconds": round(dt, 2),
            "sample": f"config 2 shapes (R50 6/6 d256 {args.size}x{args.size}), batch {B}, "
                      f"{n} timed fwd+CE+bwd steps after 1 warm-up, fp32 oracle/model.py, "
                      f"{cores} threads"}


def _traffic(family):
    """Per-launch HBM bytes of ``family`` from the committed rocprofv3 --pmc pass
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py with the gfx950 FETCH_SIZE x2
    correction), or None when no counter pass covers it."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    ent = d.get("families", {}).get(family)
    if not ent:
        return None, None
    return ent.get("bytes_per_launch"), d.get("source")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--decode-batch", type=int, default=64)
    ap.add_argument("--beam", type=int, default=5, help="beam width of the decode block (1: off)")
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU-baseline sample: timed oracle steps until this much CPU time")
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture of the step")
    ap.add_argument("--probe-steps", type=int, default=2)
    ap.add_argument("--torch-adamw", action="store_true",
                    help="torch.optim.AdamW(capturable) + clip_grad_norm_ instead of the default "
                         "retr_amd FusedAdamW (clip + AdamW kernels over flat arenas)")
    ap.add_argument("--probe-detail", default="", help="write a per-shape kernel table here")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.manual_seed(42 + rank)

    dt, loss, fam, psteps = train_bench(args, rank, world, device)
    imgs = world * args.batch * args.steps
    value = imgs / dt
    dom_key = max(fam, key=lambda k: fam[k]["ms_total"]) if fam else None
    roof = None
    if dom_key:
        d = fam[dom_key]
        achieved = d["tflops"]
        traffic, tsrc = _traffic(dom_key)
        roof = {"bound": "mfma", "kernel": dom_key,
                "kernel_symbol": probe_mod.FAMILY_SYMBOL.get(dom_key, dom_key),
                "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                "traffic_source": tsrc,
                "launches_per_step": d["launches"] // max(1, psteps),
                "avg_launch_us": round(d["ms_avg"] * 1e3, 2),
                "flops_per_launch": round(d["flops"] / max(1, d["launches"]), 1),
                "timing": "HIP events around each launch on torch's current stream (the "
                          "stream every retr kernel runs on), device spin in front so the "
                          "events bracket device time only; eager re-run of the step"}
    families = {k: {"ms_per_step": round(v["ms_total"] / psteps, 3),
                    "tflops": round(v["tflops"], 1), "launches_per_step":
                    v["launches"] // psteps} for k, v in sorted(
                        fam.items(), key=lambda kv: -kv[1]["ms_total"])}
    decode = None
    if not args.no_decode:
        res = decode_bench(args, rank, world, device)
        ddt, steps = res["greedy"]
        decode = {"metric": "greedy-decode refs/sec", "value": round(world * args.decode_batch
                                                                     / ddt, 2),
                  "unit": "refs/s", "batch_per_gpu": args.decode_batch, "steps": steps,
                  "ms_per_batch": round(ddt * 1e3, 2),
                  "config": "cfg5: ResNet-50 dilation=True 224x224, 6/6 d256, bf16, "
                            "KV-cache greedy, per-step hipGraphs (token ids equal to the "
                            "reference algorithm)"}
        for name, (bdt, bsteps) in res.items():
            if name != "greedy":
                decode[name] = {"value": round(world * args.decode_batch / bdt, 2),
                                "unit": "refs/s", "ms_per_batch": round(bdt * 1e3, 2),
                                "steps": bsteps}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
               "data": "synthetic (RefCOCO-shaped images/captions, synthetic weights)",
               "config": {"workload": "cfg2: ResNet-50 + 6-enc/6-dec d_model 256, 640x640, "
                                      f"batch {args.batch}/GPU, fwd+CE+bwd+allreduce+clip+AdamW",
                          "global_batch": world * args.batch, "seq_len": 128,
                          "parallelism": f"dp{world}"},
               "loss": round(loss, 4), "roofline": roof, "cpu_baseline": cpu,
               "launch": ("eager" if args.eager else
                          "hipGraph (whole step)" if world == 1 else
                          "hipGraph (fwd+bwd) + RCCL all-reduce + hipGraph (clip+AdamW)"),
               "optimizer": "torch.optim.AdamW" if args.torch_adamw else "FusedAdamW",
               "decode": decode, "kernel_families": families}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
