"""Drop-in for the reference loss_functions/losses.py: the pre-train branch of get_loss (losses.py:107-113,
179-182), which is what train_amos_atlas_final.py:303-304 calls for epoch < pretrain_epoch, and the refiner
loss get_loss_refine (:46-62)."""
from loss_functions.loss_partial import EDiceLoss_full, EDiceLoss_partial


def get_loss(output, cm, deep_out, target, mask=None, catlas=None, attns=None, refine_output=None, label_t=None,
             discard=0.05, confi_=0.10, aux_weight=1, weight_feature=0.1):
    """Returns (EDiceLoss_partial(C)(output, target.squeeze(1), soft_max=True, mask=mask), confi_)."""
    if len(deep_out) != 0 or refine_output is not None:
        raise NotImplementedError("get_loss: deep supervision / refiner-consistency branches are SURVEY.md §8(f) "
                                  "rows f2/f3 — not built yet")
    edice = EDiceLoss_partial(output.shape[1])
    dice_loss = edice(output, target.squeeze(1), soft_max=True, mask=mask)
    return dice_loss, confi_


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
