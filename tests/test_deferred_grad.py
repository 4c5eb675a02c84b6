"""loss.DeferredLossGrad on the CPU: the unformed hand-off reaches the producing Function as is, and every other
reader (a hook, torch.autograd.grad on the logits, a sum with a second gradient) gets the formed tensor first."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
from u3d.loss import DeferredLossGrad  # noqa: E402

LINK = object()


class _Producer(torch.autograd.Function):  # stands in for trunk._TrunkFn
    seen = []

    @staticmethod
    def forward(ctx, x):
        y = (x * 2).permute(1, 0)
        y._u3d_head_link = LINK
        return y

    @staticmethod
    def backward(ctx, g):
        unformed = isinstance(g, DeferredLossGrad) and g.link is LINK and g.unformed()
        _Producer.seen.append(unformed)
        if unformed:
            return g.payload[0].permute(1, 0) * 2  # the "fused" consumer reads the payload, never the tensor
        if isinstance(g, DeferredLossGrad):
            g = g.materialize()
        return g.permute(1, 0) * 2


class _Loss(torch.autograd.Function):  # stands in for loss._PartialLossFn
    formed = 0

    @staticmethod
    def forward(ctx, lg):
        ctx.like = (tuple(lg.shape), tuple(lg.stride()), lg.dtype, lg.device)
        ctx.link = getattr(lg, "_u3d_head_link", None)
        return lg.sum()

    @staticmethod
    def backward(ctx, g):
        shape = ctx.like[0]

        def form():
            _Loss.formed += 1
            return torch.full(shape[::-1], 3.0).permute(1, 0) * g
        return DeferredLossGrad(ctx.like, form, (torch.full(shape, 3.0) * g,), ctx.link)


def _run(extra):
    _Producer.seen.clear()
    _Loss.formed = 0
    x = torch.ones(3, 4, requires_grad=True)
    y = _Producer.apply(x)
    loss = _Loss.apply(y)
    out = {}
    if extra == "sum":
        loss = loss + y.sum()
    if extra == "hook":
        y.register_hook(lambda t: out.update(hook=float(t.sum())))
    if extra == "grad":
        (gy,) = torch.autograd.grad(loss, y)
        return float((gy * 1).sum()), out
    loss.backward()
    return x.grad, out


def test_unformed_reaches_producer():
    g, _ = _run(None)
    assert _Producer.seen == [True] and _Loss.formed == 0
    assert torch.equal(g, torch.full((3, 4), 6.0))


def test_sum_forms_first():
    g, _ = _run("sum")
    assert _Producer.seen == [False] and _Loss.formed == 1
    assert torch.equal(g, torch.full((3, 4), 8.0))


def test_hook_forms_first():
    g, out = _run("hook")
    assert out["hook"] == 36.0 and _Loss.formed == 1 and _Producer.seen == [False]
    assert torch.equal(g, torch.full((3, 4), 6.0))


def test_autograd_grad_forms():
    s, _ = _run("grad")
    assert s == 36.0 and _Loss.formed == 1 and _Producer.seen == []
