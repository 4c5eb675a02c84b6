"""Training data path on the device.

* ``crop_patch``: AMOSDataSet_newatlas.__getitem__'s tensor work (MOTSDataset.py:355-384): pad to crop + 5 (zeros),
  truncate (:171-186: CT clipped to [-325, 325] / 325 for case ids < 500, MRI z-scored over the padded volume),
  the random crop (offsets drawn with np.random in the reference's order b, c, a) and the (H, W, D) -> (D, H, W)
  transpose — one device pass per tensor (u3d_crop_transpose; the MRI statistics by u3d_volume_stats).
* ``train_transform``: my_collate's batchgenerators transforms (get_train_transform, :33-52) with their published
  parameters: Gaussian noise (p 0.1), Gaussian blur (sigma U(0.5, 1), per channel p 0.5, p 0.2), multiplicative
  brightness U(0.75, 1.25) (p 0.15), additive brightness N(0, 0.1) (per channel p 0.5, p 0.15), contrast
  (0.75, 1.25), preserve range (p 0.15). Decisions and parameters are drawn on the host with numpy; the kernels apply
  them. batchgenerators is not installed here, so the exact draw sequence is unpinned (each applied operation is
  pinned against numpy / scipy restatements in tests/test_gpu_data.py); the noise uses a counter-based device RNG.
"""
import math

import numpy as np
import torch

from . import ops
from ._lib import call, query

MODE_COPY, MODE_CT, MODE_MRI = 0, 1, 2


def volume_stats(x, count=None):
    """[mean, population std, min, max] of a device fp32 tensor extended by (count - numel) zeros (fp64, fixed
    order)."""
    x = x.float().contiguous()
    out = torch.empty(4, dtype=torch.float32, device=x.device)
    ws = ops.WS.get(query("u3d_volume_stats_ws_bytes"), x.device, slot=11)
    call("u3d_volume_stats", x.data_ptr(), x.numel(), int(count or x.numel()), out.data_ptr(), ws.data_ptr(),
         ops._stream())
    return out


def crop_transpose(src, offsets, crop, mode=MODE_COPY, stats=None):
    """src [C, H, W, D] (or [H, W, D]) fp32 device; offsets (b, c, a); crop (ch, cw, cd) -> [C, cd, ch, cw]."""
    ops.require_device(src)
    s = src.float().contiguous()
    if s.dim() == 3:
        s = s.unsqueeze(0)
    C, sh, sw, sd = s.shape
    ch, cw, cd = crop
    out = torch.empty((C, cd, ch, cw), dtype=torch.float32, device=s.device)
    call("u3d_crop_transpose", s.data_ptr(), C, sh, sw, sd, int(offsets[0]), int(offsets[1]), int(offsets[2]), ch, cw,
         cd, mode, stats.data_ptr() if stats is not None else None, out.data_ptr(), ops._stream())
    return out


def crop_patch(image, label, catlas, name, crop_size, usage="train", rng=np.random):
    """image / label [H, W, D], catlas [13, H, W, D] device tensors as read (sitk arrays); crop_size = (d, h, w) as
    the dataset's (crop_d, crop_h, crop_w). Returns image [1, D, H, W], label [1, D, H, W], catlas [13, D, H, W]."""
    cd, ch, cw = crop_size
    H, W, D = image.shape
    ph, pw, pd = max(H, ch + 5), max(W, cw + 5), max(D, cd + 5)   # pad_image to crop + 5 (zeros)
    mri = float(name) >= 500                                     # truncate(image, name), :177
    stats = None
    if mri:  # z-score over the PADDED volume: the padding zeros count, as np.mean / np.std see them
        stats = volume_stats(image, ph * pw * pd)
    if usage == "train":
        b = rng.randint(ph - ch)
        c = rng.randint(pw - cw)
        a = rng.randint(pd - cd)
        out_hw = (ch, cw, cd)
    else:
        b = c = a = 0
        out_hw = (ph, pw, pd)
    img = crop_transpose(image, (b, c, a), out_hw, MODE_MRI if mri else MODE_CT, stats)
    lab = crop_transpose(label, (b, c, a), out_hw)
    cat = crop_transpose(catlas, (b, c, a), out_hw) if catlas is not None else None
    return img, lab, cat


def gaussian_kernel1d(sigma, truncate=4.0):
    """scipy.ndimage's 1-D Gaussian (order 0): radius int(truncate * sigma + 0.5), normalised."""
    r = int(truncate * float(sigma) + 0.5)
    xs = np.arange(-r, r + 1, dtype=np.float64)
    k = np.exp(-0.5 / (sigma * sigma) * xs ** 2)
    return (k / k.sum()).astype(np.float32), r


def gaussian_blur(x, sigma):
    """scipy.ndimage.gaussian_filter(x, sigma) (mode 'reflect', truncate 4) of a [D, H, W] device volume, three
    separable passes."""
    w, r = gaussian_kernel1d(sigma)
    wt = torch.from_numpy(w).to(x.device)
    cur = x.float().contiguous()
    D, H, W = cur.shape
    for outer, L, inner in ((1, D, H * W), (D, H, W), (D * H, W, 1)):
        nxt = torch.empty_like(cur)
        call("u3d_aug_blur_axis", cur.data_ptr(), nxt.data_ptr(), outer, L, inner, wt.data_ptr(), r, ops._stream())
        cur = nxt
    return cur


def train_transform(image, rng=np.random, seed=None):
    """my_collate's intensity transforms on a device batch [B, C, D, H, W] (in place where the reference is).
    Returns the batch and a log of the applied operations (for tests / reproducibility)."""
    ops.require_device(image)
    x = image.float().contiguous()
    B, C = x.shape[:2]
    log = []
    base = int(seed if seed is not None else rng.randint(0, 2 ** 31 - 1))
    for b in range(B):                                   # GaussianNoiseTransform(p_per_sample=0.1)
        if rng.uniform() < 0.1:
            var = rng.uniform(0.0, 0.1)
            call("u3d_aug_noise", x[b].data_ptr(), x[b].numel(), float(var), (base * 1000003 + b) & (2 ** 64 - 1),
                 ops._stream())
            log.append(("noise", b, var))
    for b in range(B):                                   # GaussianBlurTransform((0.5, 1), p_ch 0.5, p 0.2)
        if rng.uniform() < 0.2:
            for c in range(C):
                if rng.uniform() < 0.5:
                    sigma = rng.uniform(0.5, 1.0)
                    x[b, c].copy_(gaussian_blur(x[b, c], sigma))
                    log.append(("blur", b, c, sigma))
    for b in range(B):                                   # BrightnessMultiplicativeTransform((0.75, 1.25), p 0.15)
        if rng.uniform() < 0.15:
            for c in range(C):
                m = rng.uniform(0.75, 1.25)
                call("u3d_aug_affine", x[b, c].data_ptr(), x[b, c].numel(), float(m), 0.0, ops._stream())
                log.append(("mul", b, c, m))
    for b in range(B):                                   # BrightnessTransform(0, 0.1, per channel, p_ch 0.5, p 0.15)
        if rng.uniform() < 0.15:
            for c in range(C):
                if rng.uniform() < 0.5:
                    a = rng.normal(0.0, 0.1)
                    call("u3d_aug_affine", x[b, c].data_ptr(), x[b, c].numel(), 1.0, float(a), ops._stream())
                    log.append(("add", b, c, a))
    for b in range(B):                                   # ContrastAugmentationTransform((0.75, 1.25), p 0.15)
        if rng.uniform() < 0.15:
            for c in range(C):
                f = rng.uniform(0.75, 1.0) if rng.uniform() < 0.5 else rng.uniform(1.0, 1.25)
                st = volume_stats(x[b, c])
                call("u3d_aug_contrast", x[b, c].data_ptr(), x[b, c].numel(), float(f), st.data_ptr(), 1,
                     ops._stream())
                log.append(("contrast", b, c, f))
    return x, log
