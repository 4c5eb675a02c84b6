"""Drop-in for the reference loss_functions/losses.py: the pre-train branch of get_loss (losses.py:107-113,
179-182), which is what train_amos_atlas_final.py:303-304 calls for epoch < pretrain_epoch."""
from loss_functions.loss_partial import EDiceLoss_partial


def get_loss(output, cm, deep_out, target, mask=None, catlas=None, attns=None, refine_output=None, label_t=None,
             discard=0.05, confi_=0.10, aux_weight=1, weight_feature=0.1):
    """Returns (EDiceLoss_partial(C)(output, target.squeeze(1), soft_max=True, mask=mask), confi_)."""
    if len(deep_out) != 0 or refine_output is not None:
        raise NotImplementedError("get_loss: deep supervision / refiner-consistency branches are SURVEY.md §8(f) "
                                  "rows f2/f3 — not built yet")
    edice = EDiceLoss_partial(output.shape[1])
    dice_loss = edice(output, target.squeeze(1), soft_max=True, mask=mask)
    return dice_loss, confi_


def get_loss_refine(*a, **k):
    raise NotImplementedError("get_loss_refine: refiner loss, SURVEY.md §8(f) row f3 — not built yet")
