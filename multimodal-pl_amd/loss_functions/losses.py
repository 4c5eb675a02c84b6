"""Drop-in for the reference loss_functions/losses.py: get_loss — the pre-train branch (losses.py:107-113,
179-182, train_amos_atlas_final.py:303-304) and the refiner-consistency branch over the feam3 attention maps
(:131-178, train_amos_atlas_final.py:312) — and the refiner loss get_loss_refine (:46-62)."""
import torch
import torch.nn.functional as F
from torch.nn.modules.loss import _WeightedLoss

from loss_functions.loss_partial import EDiceLoss_full, EDiceLoss_partial


def get_loss(output, cm, deep_out, target, mask=None, catlas=None, attns=None, refine_output=None, label_t=None,
             discard=0.05, confi_=0.10, aux_weight=1, weight_feature=0.1):
    """EDiceLoss_partial(C)(output, target.squeeze(1), soft_max=True, mask=mask); with ``refine_output`` plus the
    consistency term: masked soft Dice of every attention map (sigmoid) and of softmax(output)[:, 1:] against the
    refiner's confident foreground for the organs label_t marks unsupervised (u3d.loss.consistency_aux, one fused
    pass). ``refine_label`` (:134-157) is never read by the reference and is not built; ``refine_output`` carries
    no gradient (the driver computes it under no_grad, train_amos_atlas_final.py:285-287). Returns (loss, 0.10)."""
    if len(deep_out) != 0:
        raise NotImplementedError("get_loss: the deep_out branch (losses.py:119-129) is never used by the driver "
                                  "(train_amos_atlas_final.py:304, 312 pass []) and is not built")
    edice = EDiceLoss_partial(output.shape[1])
    dice_loss = edice(output, target.squeeze(1), soft_max=True, mask=mask)
    if refine_output is None:
        return dice_loss, confi_
    from u3d import loss as L
    if not torch.is_tensor(label_t):
        label_t = torch.tensor(label_t, dtype=torch.float32)
    aux = L.consistency_aux(output, list(attns), refine_output, label_t, weight_feature, confi=0.10)
    return dice_loss + aux * aux_weight, 0.10


def get_loss_refine(output, label, dlist, aug_mask=1):
    """Reference losses.py:46-62: sum over the refiner's samples of EDiceLoss_full(2) (uce=False) against the
    binary mask of that sample's organ (label == l + 1); with aug_mask > 1 the batch holds aug_mask copies."""
    from u3d import ops
    ops.require_device(output, label)
    loss = 0.
    cedice = EDiceLoss_full(2)
    reps = aug_mask if aug_mask > 1 else 1
    for kk in range(reps):
        start = kk * len(dlist)
        for idx, l in enumerate(dlist):
            loss += cedice(output[start + idx:start + idx + 1], (label == (l + 1)).squeeze(1), uce=False)
    return loss


def make_partial_target(labels, sup_mask):
    """train_amos_atlas_final.py:252-255: cmask = labels with organs 1..13 the dataset does not annotate (mask[l]
    == 0) set to background, one device pass (u3d_partial_target) instead of 13 masked writes."""
    from u3d import ops
    return ops.partial_target(labels, sup_mask, 1, 13).reshape(labels.shape)


class SmoothCrossEntropyLoss(_WeightedLoss):
    """Reference losses.py:441-469 — the style discriminator's loss (the discriminators are out of scope, SURVEY
    §2; this tiny [B, K] loss is kept so the driver's import line and its calls work): cross entropy against
    label-smoothed one-hot targets (smoothing / (K-1) off-target), optional class weights, mean / sum / none."""

    def __init__(self, weight=None, reduction="mean", smoothing=0.):
        super().__init__(weight=weight, reduction=reduction)
        self.smoothing = smoothing
        self.weight = weight
        self.reduction = reduction

    def k_one_hot(self, targets, n_classes, smoothing=0.0):
        with torch.no_grad():
            t = torch.full((targets.size(0), n_classes), smoothing / (n_classes - 1), device=targets.device)
            return t.scatter_(1, targets.data.unsqueeze(1), 1. - smoothing)

    def reduce_loss(self, loss):
        return loss.mean() if self.reduction == "mean" else loss.sum() if self.reduction == "sum" else loss

    def forward(self, inputs, targets):
        assert 0 <= self.smoothing < 1
        targets = self.k_one_hot(targets, inputs.size(-1), self.smoothing)
        log_preds = F.log_softmax(inputs, -1)
        if self.weight is not None:
            log_preds = log_preds * self.weight.unsqueeze(0)
        return self.reduce_loss(-(targets * log_preds).sum(dim=-1))


def bce_loss(y_pred, y_label):
    """Reference losses.py:471-475: SmoothCrossEntropyLoss against a constant class label for the whole batch."""
    y = torch.full((y_pred.shape[0],), float(y_label), device=y_pred.device).long()
    return SmoothCrossEntropyLoss()(y_pred, y)
