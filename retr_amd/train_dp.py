"""Data-parallel training launcher: the reference's main.py training loop (main.py:15-103) with
one process per GPU (``torchrun --nproc-per-node N -m retr_amd.train_dp``, RCCL over xGMI).

Differences from main.py, all forced by data parallelism or the MI355X optimizer path:
  * ``DistributedSampler`` (shuffle, ``set_epoch`` per epoch, drop_last) + ``BatchSampler``
    replace ``RandomSampler`` + ``BatchSampler`` (main.py:51-60); ``config.batch_size`` is the
    per-GPU batch, the global batch is ``world_size`` times it;
  * rank 0's initial weights are broadcast (the reference seeds ``config.seed + rank``,
    main.py:19-21: the same is kept for the data-side RNGs);
  * the optimizer is ``FusedAdamW`` over the same two parameter groups (main.py:30-39) and the
    gradients are averaged in place on its arena by ``GradSync`` (retr_amd/ddp.py);
  * the epoch loss is averaged over ranks; the validation loss is the reference's evaluate()
    over the whole validation set (SequentialSampler, main.py:52) run on rank 0 and broadcast;
    rank 0 prints and writes checkpoints (train_utils/checkpoints.py format);
  * a non-finite loss on any rank stops every rank (engine.train_one_epoch agrees on it with
    one all-reduce), so no rank is left waiting in a collective.
The CIDEr evaluation (eval_model, nlgeval + BERT tokenizer) and early stopping stay with the
caller: they need network-fetched assets outside the hot path.
"""
import os

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import BatchSampler, DataLoader, DistributedSampler


def dist_timeout():
    """Collective timeout of the process group: ``RETR_DIST_TIMEOUT_S`` seconds, default one
    hour.  The validation pass runs on rank 0 alone while every other rank waits in the
    broadcast of its loss (``_from_rank0``), so the timeout must exceed one full ``evaluate()``
    over the validation set -- NCCL's 10-minute default does not on a large set."""
    import datetime
    return datetime.timedelta(seconds=float(os.environ.get("RETR_DIST_TIMEOUT_S", "3600")))


def init_distributed():
    """Process group from the torchrun environment (RANK/WORLD_SIZE/MASTER_*), RCCL when a GPU
    is visible.  Returns (rank, world_size, local_rank); (0, 1, 0) without torchrun."""
    if "RANK" in os.environ and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", 0))
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend, timeout=dist_timeout())
    if not dist.is_initialized():
        return 0, 1, 0
    return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", 0))


def build_loaders(config, dataset_train, dataset_val, rank, world):
    sampler_train = DistributedSampler(dataset_train, num_replicas=world, rank=rank,
                                       shuffle=True, seed=config.seed, drop_last=True)
    batch_sampler_train = BatchSampler(sampler_train, config.batch_size, drop_last=True)
    loader_train = DataLoader(dataset_train, batch_sampler=batch_sampler_train,
                              num_workers=config.num_workers)
    loader_val = None
    if dataset_val is not None and rank == 0:
        # the reference's own validation loader (main.py:52,61-62), on rank 0 only: a sharded
        # DistributedSampler would pad the set with repeats and change the batch partition,
        # so the rank-averaged loss would not be evaluate()'s value over the exact val set
        loader_val = DataLoader(dataset_val, config.batch_size,
                                sampler=torch.utils.data.SequentialSampler(dataset_val),
                                drop_last=False, num_workers=config.num_workers)
    return loader_train, loader_val, sampler_train


def _from_rank0(v, device, world):
    """Rank 0's value on every rank (the validation loss is computed on rank 0 only)."""
    if world == 1:
        return v
    t = torch.tensor([float("nan") if v is None else float(v)], dtype=torch.float64,
                     device=device)
    dist.broadcast(t, 0)
    return t.item()


def _mean_over_ranks(v, device, world):
    if world == 1:
        return v
    t = torch.tensor([float(v)], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return t.item() / world


def main(config, dataset_train, dataset_val=None, epochs=None, checkpoint_dir=None):
    """Train for ``epochs`` (default config.epochs - config.start_epoch); returns the list of
    (epoch, train_loss, val_loss) averaged over ranks."""
    from .ddp import GradSync, broadcast_parameters
    from .engine import evaluate, train_one_epoch
    from .models import caption
    from .optim import FusedAdamW
    from .train_utils.checkpoints import save_ckp

    rank, world, local = init_distributed()
    device = torch.device(f"cuda:{local}" if world > 1 else config.device)
    seed = config.seed + rank
    torch.manual_seed(seed)
    np.random.seed(seed)

    model, criterion = caption.build_model(config)
    model.to(device)
    distributed = dist.is_initialized()
    if distributed:
        broadcast_parameters(model)
    if rank == 0:
        print(f"Number of params: {sum(p.numel() for p in model.parameters() if p.requires_grad)}")
    param_dicts = [
        {"params": [p for n, p in model.named_parameters()
                    if "backbone" not in n and p.requires_grad]},
        {"params": [p for n, p in model.named_parameters()
                    if "backbone" in n and p.requires_grad], "lr": config.lr_backbone},
    ]
    optimizer = FusedAdamW(param_dicts, lr=config.lr, weight_decay=config.weight_decay)
    lr_scheduler = torch.optim.lr_scheduler.StepLR(optimizer, config.lr_drop)
    grad_sync = None
    if distributed:
        grad_sync = GradSync([p for p in model.parameters() if p.requires_grad],
                             bucket_mb=getattr(config, "grad_bucket_mb", 64),
                             optimizer=optimizer)
    loader_train, loader_val, sampler_train = build_loaders(config, dataset_train, dataset_val,
                                                            rank, world)
    history = []
    last = config.start_epoch + epochs if epochs is not None else config.epochs
    for epoch in range(config.start_epoch, last):
        sampler_train.set_epoch(epoch)
        if rank == 0:
            print(f"Epoch: {epoch}")
        epoch_loss = train_one_epoch(model, criterion, loader_train, optimizer, device, epoch,
                                     config.clip_max_norm, grad_sync)
        lr_scheduler.step()
        epoch_loss = _mean_over_ranks(epoch_loss, device, world)
        val_loss = None
        if dataset_val is not None:
            if loader_val is not None:
                val_loss = evaluate(model, criterion, loader_val, device)
            val_loss = _from_rank0(val_loss, device, world)
        if rank == 0:
            print(f"Training Loss: {epoch_loss}")
            if val_loss is not None:
                print(f"Validation Loss: {val_loss}")
            if checkpoint_dir is not None:
                os.makedirs(checkpoint_dir, exist_ok=True)
                save_ckp(epoch, model, optimizer, lr_scheduler, train_loss=epoch_loss,
                         val_loss=val_loss, cider_score=None,
                         path=os.path.join(checkpoint_dir, f"{config.transformer_type}_"
                                           f"{config.prefix}_checkpoint_{epoch}.pth"))
        history.append((epoch, epoch_loss, val_loss))
    return history


if __name__ == "__main__":
    # synthetic RefCOCO-shaped data (the RefCOCO images / BERT tokenizer are not fetched here)
    from .configuration import Config
    from .synthetic import SyntheticRefDataset
    cfg = Config()
    n = int(os.environ.get("RETR_SYNTH_SAMPLES", "64"))
    main(cfg, SyntheticRefDataset(cfg, n, 640), SyntheticRefDataset(cfg, n // 4, 640, seed=7),
         epochs=int(os.environ.get("RETR_EPOCHS", "1")))
