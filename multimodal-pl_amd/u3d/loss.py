"""Autograd Function for the fused partial-label Dice + BCE loss (reference loss_partial.py:59-99)."""
import torch

from . import ops

MODE_SIGMOID, MODE_SOFTMAX, MODE_IDENTITY = 0, 1, 2


def ndhwc_view(x):
    """[S, C, D, H, W] -> NDHWC-contiguous [S, D, H, W, C] (free when x came from the native head)."""
    y = x.permute(0, 2, 3, 4, 1)
    return y if y.is_contiguous() else y.contiguous()


def class_weights(mask, C, device):
    """mask[0] of the reference (only the first sample's supervision vector is used, loss_partial.py:87)."""
    if mask is None:
        return torch.ones(C, dtype=torch.float32, device=device)
    w = mask[0]
    if not torch.is_tensor(w):
        w = torch.tensor(w)
    if w.numel() < C:
        raise IndexError(f"index {w.numel()} is out of bounds for dimension 0 with size {w.numel()} "
                         f"(mask[0] shorter than the {C} classes, as the reference's weight[i] would fail)")
    return w.reshape(-1)[:C].to(device=device, dtype=torch.float32)


class _PartialLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, weights, mode, uce):
        lg = ndhwc_view(logits.float())
        lab = target.float().contiguous()
        loss, sums = ops.partial_loss_fwd(lg, lab, weights, mode, uce)
        ctx.save_for_backward(lg, lab, weights, sums)
        ctx.mode, ctx.uce = mode, uce
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        lg, lab, weights, sums = ctx.saved_tensors
        go = g.reshape(1).float().contiguous()
        dl = ops.partial_loss_bwd(lg, lab, weights, sums, go, ctx.mode, ctx.uce)
        return dl.permute(0, 4, 1, 2, 3), None, None, None, None


def partial_loss(logits, target, weights, mode=MODE_SOFTMAX, uce=True):
    ops.require_device(logits, target)
    if target.shape[0] != logits.shape[0] or target.numel() * logits.shape[1] != logits.numel():
        raise AssertionError(f"predict {tuple(logits.shape)} & target {tuple(target.shape)} shape do not match")
    return _PartialLossFn.apply(logits, target, weights, mode, uce)
