"""Autograd wrapper to run one sub-module (a weight-standardised conv, a NoBottleneck block) on the native
executor when a caller uses that module on its own, outside the full trunk."""
import torch

from . import ops
from .trunk import Act, Tape, compute_dtype


class _SubFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, builder, dtype, std, names, x, *tensors):
        tape = Tape(dict(zip(names, tensors)), dtype, record=True)
        tape.std = std
        xa = Act(x.permute(0, 2, 3, 4, 1).contiguous().to(dtype))
        out = builder(tape, xa)
        ctx.tape, ctx.xa, ctx.out, ctx.names = tape, xa, out, names
        return out.t.permute(0, 4, 1, 2, 3).float()

    @staticmethod
    def backward(ctx, g):
        tape = ctx.tape
        g = g.permute(0, 2, 3, 4, 1).contiguous().to(ctx.out.t.dtype)
        tape.backward(ctx.out, g)
        dx = ctx.xa.grad
        dx = dx.float().permute(0, 4, 1, 2, 3) if dx is not None else None
        grads = [tape.pgrad.get(n) for n in ctx.names]
        return (None, None, None, None, dx, *grads)


def run(builder, x, named_params, std=True, dtype=None):
    """x: NCDHW fp32 device tensor; builder(tape, act) -> Act. Returns NCDHW fp32."""
    ops.require_device(x)
    dtype = compute_dtype(dtype)
    names = [n for n, _ in named_params]
    tensors = [p for _, p in named_params]
    return _SubFn.apply(builder, dtype, std, names, x, *tensors)
