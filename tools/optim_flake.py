"""Repeat tests/test_gpu_optim.py::test_train_steps_fused_vs_torch_optimizer's body (deterministic
mode) and print every step's two losses, to localise an intermittent mismatch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_optim import FusedAdamW, _batch, _groups, _micro_model  # noqa: E402
from retr_amd import ops  # noqa: E402
from retr_amd.engine import train_step  # noqa: E402


def main():
    ops.set_deterministic(True)
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
        cfg, m1, crit = _micro_model()
        _, m2, _ = _micro_model()
        o1 = FusedAdamW(_groups(m1, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay)
        o2 = torch.optim.AdamW(_groups(m2, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay,
                               foreach=False)
        samples, caps, cm = _batch(cfg)
        m1.train()
        m2.train()
        out = []
        for _ in range(3):
            l1 = train_step(m1, crit, samples, caps, cm, o1, 0.1)
            l2 = train_step(m2, crit, samples, caps, cm, o2, 0.1)
            out.append((l1.item(), l2.item()))
        bad = [i for i, (a, b) in enumerate(out) if abs(a - b) > 1e-6 * abs(b)]
        print(rep, "bad steps", bad, " ".join(f"{a:.7f}/{b:.7f}" for a, b in out), flush=True)


if __name__ == "__main__":
    main()
