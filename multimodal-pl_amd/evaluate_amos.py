"""Drop-in for the metric part of the reference evaluate_amos.py.

get_dice (evaluate_amos.py:128-154, atlas=None branch) runs as one fused HIP pass: per-voxel argmax of the
softmax, integer per-class counts, and the fp32 dice / sensitivity / precision averaged over samples exactly
as the reference's dice_score / senc_score / spec_score (:92-126) compute them from the counts.
dice_score / spec_score / senc_score themselves are kept as the reference's small tensor helpers.
Sliding-window inference (predict_sliding, _get_gaussian, :184-279) keeps the
reference's tiling, multi-net averaging and flip test-time augmentation, but accumulates on the device
(libu3d window kernels, fp32) instead of copying every tile's prediction to float64 host arrays.
"""
import math

import numpy as np
import torch
import torch.distributed as dist

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


def get_dice2(preds, labels, t_id, atlas=None, num_class=13):
    """Reference evaluate_amos.py:156-182 (the refiner's metric, train_amos_atlas_final.py:294): preds = the
    refiner output [num_class organs, 2, D, H, W]; organ l's binary prediction argmax(softmax(preds[l])) == 1 is
    scored against labels == l+1. One fused pass (u3d_dice_metric_binary). Returns (dices, senc, spec, argmax)."""
    if atlas is not None:
        raise NotImplementedError("get_dice2 atlas branch (evaluate_amos.py:170-180) is not on the native path")
    from u3d._lib import call
    from u3d.loss import _voxel_strides
    ops.require_device(preds, labels)
    if preds.shape[0] < num_class or preds.shape[1] != 2:
        raise AssertionError("predict & target batch size don't match")  # dice_score on an empty slice
    ref, (rsn, rsc, rsv) = _voxel_strides(preds.float(), 2)
    V = ref[0, 0].numel()
    lab = labels.float().reshape(-1).contiguous()
    if lab.numel() != V:
        raise RuntimeError(f"get_dice2: labels {tuple(labels.shape)} vs prediction volume {tuple(preds.shape[2:])}")
    counts = torch.empty((num_class, 3), dtype=torch.int64, device=preds.device)
    metrics = torch.empty((num_class, 3), dtype=torch.float32, device=preds.device)
    am = torch.empty((preds.shape[0],) + tuple(preds.shape[2:]), dtype=torch.int64, device=preds.device)
    call("u3d_dice_metric_binary", ref.data_ptr(), num_class, V, rsn, rsc, rsv, lab.data_ptr(), counts.data_ptr(),
         metrics.data_ptr(), am.data_ptr(), ops._stream())
    if preds.shape[0] > num_class:  # the reference's argmax covers every organ of the batch
        call("u3d_dice_metric_binary", ref.data_ptr(), preds.shape[0], V, rsn, rsc, rsv, lab.data_ptr(),
             torch.empty((preds.shape[0], 3), dtype=torch.int64, device=preds.device).data_ptr(),
             torch.empty((preds.shape[0], 3), dtype=torch.float32, device=preds.device).data_ptr(), am.data_ptr(),
             ops._stream())
    dices = [metrics[l, 0] for l in range(num_class)]
    senc = [metrics[l, 1] for l in range(num_class)]
    spec = [metrics[l, 2] for l in range(num_class)]
    return dices, senc, spec, am


def _gaussian_profiles(patch_size, sigma_scale=1.0 / 8):
    """The 1-D factors of _get_gaussian (evaluate_amos.py:184-197): scipy.ndimage.gaussian_filter (truncate 4.0,
    mode 'constant') of a centred delta is the product of three normalised 1-D kernels; each factor is scaled
    to max 1 (so the map's max is 1) and the map's zeros become its minimum non-zero value ``gmin``."""
    profs, mins = [], []
    for n in patch_size:
        sigma = n * sigma_scale
        radius = int(4.0 * sigma + 0.5)
        xs = np.arange(-radius, radius + 1, dtype=np.float64)
        k = np.exp(-0.5 * (xs / sigma) ** 2)
        k /= k.sum()
        c = n // 2
        prof = np.zeros(n, dtype=np.float64)
        for i in range(n):
            if -radius <= i - c <= radius:
                prof[i] = k[i - c + radius]
        prof /= prof.max()
        profs.append(prof)
        mins.append(prof[prof > 0].min())
    return profs, float(np.float32(np.prod(mins)))


def _get_gaussian(patch_size, sigma_scale=1.0 / 8):
    """The full importance map (float32, as the reference returns it) — for inspection; predict_sliding uses the
    separable factors on the device."""
    (pd, ph, pw), gmin = _gaussian_profiles(patch_size, sigma_scale)
    g = (pd[:, None, None] * ph[None, :, None] * pw[None, None, :]).astype(np.float32)
    g[g == 0] = gmin
    return g


def _as_ndhwc(pred):
    pred = pred[0] if isinstance(pred, (tuple, list)) else pred
    p = pred.float().permute(0, 2, 3, 4, 1)
    return p if p.is_contiguous() else p.contiguous()


def tile_plan(image_size, tile_size):
    """The reference's tile sequence (evaluate_amos.py:205-236): overlap 1/4, ceil strides, tiles clamped to the
    volume. Returns [(d1, d2, y1, y2, x1, x2)] in the reference's dep/row/col order."""
    overlap = 1 / 4
    strideHW = math.ceil(tile_size[1] * (1 - overlap))
    strideD = math.ceil(tile_size[0] * (1 - overlap))
    D, H, W = image_size[-3], image_size[-2], image_size[-1]
    tile_deps = int(math.ceil((D - tile_size[0]) / strideD) + 1)
    tile_rows = int(math.ceil((H - tile_size[1]) / strideHW) + 1)
    tile_cols = int(math.ceil((W - tile_size[2]) / strideHW) + 1)
    plan = []
    for dep in range(tile_deps):
        for row in range(tile_rows):
            for col in range(tile_cols):
                d1, x1, y1 = int(dep * strideD), int(col * strideHW), int(row * strideHW)
                d2 = min(d1 + tile_size[0], D)
                x2 = min(x1 + tile_size[2], W)
                y2 = min(y1 + tile_size[1], H)
                d1, x1, y1 = max(int(d2 - tile_size[0]), 0), max(int(x2 - tile_size[2]), 0), max(int(y2 - tile_size[1]), 0)
                plan.append((d1, d2, y1, y2, x1, x2))
    return plan


def shard_tiles(plan, rank, world):
    """Tiles are independent: rank r takes tiles r, r + world, ... (round-robin keeps the ranks'
    shares within one tile of each other for any tile count)."""
    return plan[rank::world]


def predict_sliding(args, net_list, image, tile_size, classes, task_id, tta=False, group=None):
    """Reference evaluate_amos.py:198-279. Returns full_probs [N, classes, D, H, W] as a device fp32 tensor (the
    reference returns a float64 CPU tensor). With a process ``group`` of world size > 1 (one process per GPU) the
    tiles are sharded round-robin over the ranks and the weighted sums / counts are summed with one all-reduce
    each (RCCL), then normalised: every rank returns the full volume."""
    from u3d import _lib
    dev = next(net_list[0].parameters()).device
    img_all = torch.as_tensor(image).to(device=dev, dtype=torch.float32)
    ops.require_device(img_all)
    image_size = img_all.shape
    N, D, H, W = image_size[0], image_size[2], image_size[3], image_size[4]
    plan = tile_plan(image_size, tile_size)
    world = 1
    if group is not None or (dist.is_available() and dist.is_initialized() and getattr(args, "shard_tiles", False)):
        world = dist.get_world_size(group)
        plan = shard_tiles(plan, dist.get_rank(group), world)
    full = torch.zeros((N, classes, D, H, W), dtype=torch.float32, device=dev)
    count = torch.zeros((N, D, H, W), dtype=torch.float32, device=dev)
    (pd, ph, pw), gmin = _gaussian_profiles(tile_size)
    gd, gh, gw = (torch.tensor(p, dtype=torch.float32, device=dev) for p in (pd, ph, pw))
    flip_sets = [()] + ([(2,), (3,), (4,), (2, 3), (2, 4), (3, 4), (2, 3, 4)] if tta else [])
    scale = 1.0 / (len(net_list) * len(flip_sets))
    for d1, d2, y1, y2, x1, x2 in plan:
        img = img_all[:, :, d1:d2, y1:y2, x1:x2].contiguous()
        first = 1
        for dims in flip_sets:
            inp = torch.flip(img, dims) if dims else img
            flags = sum({2: 1, 3: 2, 4: 4}[d] for d in dims)
            for net in net_list:
                p = _as_ndhwc(net(inp, task_id))
                if p.shape[-1] != classes or tuple(p.shape[1:4]) != (d2 - d1, y2 - y1, x2 - x1):
                    raise ValueError(f"predict_sliding: prediction {tuple(p.shape)} does not match the tile "
                                     f"({d2 - d1}, {y2 - y1}, {x2 - x1}) x {classes} classes")
                _lib.call("u3d_window_accumulate", p.data_ptr(), N, classes, d2 - d1, y2 - y1, x2 - x1,
                          gd.data_ptr(), gh.data_ptr(), gw.data_ptr(), float(gmin), float(scale),
                          full.data_ptr(), count.data_ptr(), D, H, W, d1, y1, x1, flags, first, ops._stream())
                first = 0
    if world > 1:
        dist.all_reduce(full, group=group)
        dist.all_reduce(count, group=group)
    _lib.call("u3d_window_normalize", full.data_ptr(), count.data_ptr(), N, classes, D * H * W, ops._stream())
    return full
