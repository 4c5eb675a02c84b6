"""Drop-in for the metric part of the reference evaluate_amos.py.

get_dice (evaluate_amos.py:128-154, atlas=None branch) runs as one fused HIP pass: per-voxel argmax of the
softmax, integer per-class counts, and the fp32 dice / sensitivity / precision averaged over samples exactly
as the reference's dice_score / senc_score / spec_score (:92-126) compute them from the counts.
dice_score / spec_score / senc_score themselves are kept as the reference's small tensor helpers.
Sliding-window inference (predict_sliding, _get_gaussian) is SURVEY.md §8(f) row f1.
"""
import torch

from u3d import ops
from u3d.loss import ndhwc_view


def dice_score(preds, labels):
    assert preds.shape[0] == labels.shape[0], "predict & target batch size don't match"
    predict = preds.contiguous().view(preds.shape[0], -1)
    target = labels.contiguous().view(labels.shape[0], -1)
    num = torch.sum(torch.mul(predict, target), dim=1)
    den = torch.sum(predict, dim=1) + torch.sum(target, dim=1) + 1
    return (2 * num / den).mean()


def spec_score(preds, labels):
    assert preds.shape[0] == labels.shape[0], "predict & target batch size don't match"
    predict = preds.contiguous().view(preds.shape[0], -1)
    target = labels.contiguous().view(labels.shape[0], -1)
    num = torch.sum(torch.mul(predict, target), dim=1)
    return (num / (torch.sum(predict, dim=1) + 1)).mean()


def senc_score(preds, labels):
    assert preds.shape[0] == labels.shape[0], "predict & target batch size don't match"
    predict = preds.contiguous().view(preds.shape[0], -1)
    target = labels.contiguous().view(labels.shape[0], -1)
    num = torch.sum(torch.mul(predict, target), dim=1)
    return (num / (torch.sum(target, dim=1) + 1)).mean()


def get_dice(preds, labels, t_id, atlas=None, num_class=13):
    """Returns (dices, senc, spec, argmax) like the reference: three lists of 0-dim tensors + the argmax map."""
    if atlas is not None:
        raise NotImplementedError("get_dice atlas branch (evaluate_amos.py:144-151) is not on the native path")
    ops.require_device(preds, labels)
    lg = ndhwc_view(preds.float())
    lab = labels.float().reshape(preds.shape[0], -1).contiguous()
    metrics, _, am = ops.dice_metric(lg, lab, num_class, want_argmax=True)
    dices = [metrics[l, 0] for l in range(num_class)]
    senc = [metrics[l, 1] for l in range(num_class)]
    spec = [metrics[l, 2] for l in range(num_class)]
    return dices, senc, spec, am


def predict_sliding(*a, **k):
    raise NotImplementedError("predict_sliding: sliding-window inference is SURVEY.md §8(f) row f1 — next round")
