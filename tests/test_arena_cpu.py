"""Gradient-arena hand-out semantics (retr_amd/optim.py) on the CPU: the backward Functions
write parameter gradients into zeroed arena slots that autograd adopts without a copy, and
every other case (several contributors, accumulation across backward passes, resets) gives
exactly autograd's default result."""
import torch

from retr_amd.optim import _GradArena, grad_buffer


class _MatmulW(torch.autograd.Function):
    """y = x w^T with the weight gradient produced through grad_buffer (as ops.py does)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return x @ w.detach().t()

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        dw, _ = grad_buffer(ctx.w)
        dw += dy.t() @ x
        return None, dw


def _setup():
    G = torch.zeros(64)
    arena = _GradArena(G)
    p = torch.nn.Parameter(torch.randn(4, 4))
    p._retr_grad_view = G[16:32].view(4, 4)
    p._retr_arena = arena
    x = torch.randn(3, 4)
    ref = torch.ones(3, 4).t() @ x
    return arena, p, x, ref


def test_arena_gradient_adopted_without_copy():
    arena, p, x, ref = _setup()
    _MatmulW.apply(x, p).sum().backward()
    assert p.grad.data_ptr() == p._retr_grad_view.data_ptr()
    torch.testing.assert_close(p.grad, ref)


def test_arena_several_contributors_and_accumulation():
    arena, p, x, ref = _setup()
    (_MatmulW.apply(x, p).sum() + 2 * _MatmulW.apply(x, p).sum()).backward()
    torch.testing.assert_close(p.grad, 3 * ref)
    _MatmulW.apply(x, p).sum().backward()          # no zero_grad: autograd accumulates
    torch.testing.assert_close(p.grad, 4 * ref)
    p.grad = None
    arena.reset()                                  # what FusedAdamW.zero_grad does
    _MatmulW.apply(x, p).sum().backward()
    torch.testing.assert_close(p.grad, ref)
    assert p.grad.data_ptr() == p._retr_grad_view.data_ptr()


def test_arena_stale_slot_never_reused_without_reset():
    arena, p, x, ref = _setup()
    _MatmulW.apply(x, p).sum().backward()
    p.grad = None                                  # e.g. model.zero_grad(): arena not reset
    _MatmulW.apply(x, p).sum().backward()
    torch.testing.assert_close(p.grad, ref)        # fresh buffer, not the dirty slot
