"""Drop-in for the reference loss_functions/loss_partial.py (partial-label Dice + BCE).

DiceLoss / EDiceLoss_partial keep the reference's names, constructor and forward signatures and its
quirks (loss_partial.py:10-99): only ``mask[0]`` weights the whole batch, the per-class dice is summed over
all samples and voxels together, the sum is divided by C (not by the weight sum), an all-zero mask gives
loss 0, BCE is torch's BCELoss (mean over S*V, logs clamped at -100). The whole loss is one fused HIP pass
(forward: per-class sums; backward: one elementwise pass) — u3d.loss.

``autocast`` is referenced but never imported by the reference (:4 commented, :90 used), so uce=True raises
NameError there; here the fp32 no-op it was meant to be is applied.
"""
import torch
from torch import nn

from u3d import loss as _L


class DiceLoss(nn.Module):
    """Reference loss_partial.py:10-57; inputs are probabilities."""

    def __init__(self, n_classes):
        super().__init__()
        self.n_classes = n_classes

    def _one_hot_encoder(self, input_tensor):
        return torch.cat([(input_tensor == i).unsqueeze(1) for i in range(self.n_classes)], dim=1).float()

    def forward(self, inputs, target, weight=None, softmax=True, mask=None):
        if mask is not None:
            raise NotImplementedError("DiceLoss spatial mask argument is not on the native path")
        assert inputs.shape[1] == self.n_classes, "predict & target shape do not match"
        w = _L.class_weights(None if weight is None else [weight], self.n_classes, inputs.device)
        return _L.partial_loss(inputs, target, w, mode=_L.MODE_IDENTITY, uce=False)


class EDiceLoss_partial(nn.Module):
    """Reference loss_partial.py:59-99."""

    def __init__(self, n_classes):
        super().__init__()
        self.labels = ["ET", "TC", "WT"] + ["a"] * 20
        self.device = "cpu"
        self.n_classes = n_classes
        self.diceloss = DiceLoss(n_classes=n_classes)
        self.bce = nn.BCELoss()

    def forward(self, inputs, target, mask=None, soft_max=True, uce=True):
        C = inputs.shape[1]
        w = _L.class_weights(mask, C, inputs.device)
        mode = _L.MODE_SOFTMAX if soft_max else _L.MODE_SIGMOID
        return _L.partial_loss(inputs, target, w, mode=mode, uce=bool(uce))


class EDiceLoss_full(nn.Module):
    """Reference loss_partial.py:102-135: soft Dice over all classes (DiceLoss, weights 1) of softmax (or sigmoid)
    probabilities + nn.CrossEntropyLoss of the logits when uce. One fused pass (uce=2: cross-entropy mode)."""

    def __init__(self, n_classes):
        super().__init__()
        self.labels = ["ET", "TC", "WT"] + ["a"] * 20
        self.device = "cpu"
        self.n_classes = n_classes
        self.diceloss = DiceLoss(n_classes=n_classes)
        self.bce = nn.BCELoss()
        self.mce = nn.CrossEntropyLoss()

    def forward(self, inputs, target, logits="softmax", uce=True):
        if logits == "extend":
            raise NotImplementedError("EDiceLoss_full(logits='extend') is not on the native path")
        C = inputs.shape[1]
        assert C == self.n_classes, "predict & target shape do not match"
        w = torch.ones(C, dtype=torch.float32, device=inputs.device)
        if logits == "softmax":
            return _L.partial_loss(inputs, target, w, mode=_L.MODE_SOFTMAX, uce=2 if uce else 0)
        if uce:
            raise NotImplementedError("EDiceLoss_full: sigmoid probabilities with the cross-entropy term")
        return _L.partial_loss(inputs, target, w, mode=_L.MODE_SIGMOID, uce=0)


class EDiceLoss_full2(nn.Module):
    """Reference loss_partial.py:137-170 (binary soft Dice on sigmoid(inputs) or inputs vs a soft target over the
    mask, + BCEWithLogits when uce): one fused device pass each way (u3d_edice_full2_fwd/_bwd)."""

    def __init__(self, n_classes):
        super().__init__()
        self.labels = ["ET", "TC", "WT"] + ["a"] * 20
        self.device = "cpu"
        self.n_classes = n_classes
        self.diceloss = DiceLoss(n_classes=n_classes)

    def forward(self, inputs, target, uce=True, mask=None, sigmoid=True):
        from u3d import loss as L
        return L.edice_full2(inputs, target, uce=uce, mask=mask, sigmoid=sigmoid)
