"""Data-parallel gradient sync (retr_amd.ddp.GradSync) with world_size 2 over gloo on CPU:
DP(2 x B/2) gradients == single-process gradients of the concatenated batch."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grads(sd, names, cfg, images, mask, caps, cap_mask):
    from oracle import model as orc
    for n in names:
        sd[n].grad = None
    lo = orc.caption_forward(sd, cfg, images, mask, caps[:, :-1], cap_mask[:, :-1])
    orc.caption_loss(lo, caps[:, 1:]).backward()


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from retr_amd.ddp import GradSync
    from retr_amd.models.caption import build_model
    from retr_amd.synthetic import synthetic_captions, synthetic_images, synthetic_state_dict
    from tests.helpers import make_config
    cfg = make_config(backbone="ResNet18", hidden=64, layers=(1, 1), vocab=1000, max_pos=16,
                      ffn=128)
    model, _ = build_model(cfg)
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    sd = synthetic_state_dict(model, seed=42)
    sd = {k: (v.requires_grad_(True) if k in names else v) for k, v in sd.items()}
    images, mask = synthetic_images(4, 64, seed=1, pad_band=True)
    caps, cap_mask = synthetic_captions(4, 16, 1000, seed=2)
    # single-process reference on the full batch
    _grads(sd, names, cfg, images, mask, caps, cap_mask)
    ref = {n: sd[n].grad.clone() for n in names}
    sync = GradSync([sd[n] for n in names], bucket_mb=1)
    sl = slice(2 * rank, 2 * rank + 2)
    _grads(sd, names, cfg, images[sl], mask[sl], caps[sl], cap_mask[sl])
    sync.synchronize()
    worst = max(((sd[n].grad - ref[n]).norm() / ref[n].norm().clamp_min(1e-12)).item()
                for n in names)
    q.put((rank, worst, len(sync.buckets)))
    dist.destroy_process_group()


def test_gradsync_equals_concatenated_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, worst, nb in res:
        assert nb > 1                  # exercised multiple buckets
        assert worst < 1e-5, (rank, worst)


def _timeout_worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import bench
    bench.init_dist(rank, backend="gloo")
    t = torch.ones(1) * (rank + 1)
    dist.all_reduce(t)                          # the group works
    pg = dist.group.WORLD._get_backend(torch.device("cpu"))
    q.put((rank, pg.options._timeout.total_seconds(), t.item()))
    dist.destroy_process_group()


def test_bench_process_group_has_short_timeout():
    """bench.py's multi-rank process group (the driver's SCALE run) is created with the 2-minute
    collective timeout (bench.DIST_TIMEOUT), not the 10-minute default: a first 8-rank run that
    deadlocks fails fast.  gloo world 2 through the same init_dist the nccl path uses."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, secs, tot in res:
        assert secs == 120.0, (rank, secs)
        assert tot == 3.0
