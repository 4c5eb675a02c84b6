"""CPU restatement (plain torch fp32) of the reference hot path. TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.

Parity status: PINNED. tests/test_oracle_golden.py checks every function below against the golden vectors that
tests/golden/gen_golden.py produced by importing /root/reference in the build container.

Parameters are passed as a dict keyed exactly like the reference state_dict (e.g. ``layer1.0.conv1.weight``).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


# --------------------------------------------------------------------------------------------------- A1
def ws_weight(w: torch.Tensor) -> torch.Tensor:
    """Weight standardisation, unet3D.py:21-26: per output channel mean over (Cin,k,k,k), unbiased variance
    of the centred weight, ``+1e-12`` inside the sqrt."""
    mean = w.mean(dim=1, keepdim=True).mean(dim=2, keepdim=True).mean(dim=3, keepdim=True).mean(dim=4, keepdim=True)
    wc = w - mean
    std = torch.sqrt(torch.var(wc.reshape(w.shape[0], -1), dim=1) + 1e-12).reshape(-1, 1, 1, 1, 1)
    return wc / std


def conv(x, w, stride=1, bias=None, ws=True):
    """unet3D.py:27 / conv3x3x3 :30-35 — pad = k//2 (1 for 3^3, 0 for 1^3)."""
    k = w.shape[2]
    return F.conv3d(x, ws_weight(w) if ws else w, bias, stride, k // 2)


# --------------------------------------------------------------------------------------------- A4 / A5
def gn_relu(x, groups, gamma, beta):
    """nn.GroupNorm(G, C) (eps 1e-5, biased variance) then ReLU — unet3D.py:44-47."""
    return F.relu(F.group_norm(x, groups, gamma, beta, 1e-5))


# ------------------------------------------------------------------------------------------------- A3
def block(P, pre, x, stride, groups, ws=True):
    """NoBottleneck.forward, unet3D.py:56-73; downsample = GN -> ReLU -> 1^3 conv stride s (_make_layer :1666-1686)."""
    out = conv(gn_relu(x, groups, P[pre + "gn1.weight"], P[pre + "gn1.bias"]), P[pre + "conv1.weight"], stride, ws=ws)
    out = conv(gn_relu(out, groups, P[pre + "gn2.weight"], P[pre + "gn2.bias"]), P[pre + "conv2.weight"], 1, ws=ws)
    if pre + "downsample.0.weight" in P:
        res = conv(gn_relu(x, groups, P[pre + "downsample.0.weight"], P[pre + "downsample.0.bias"]),
                   P[pre + "downsample.2.weight"], stride, ws=ws)
    else:
        res = x
    return out + res


def layer(P, name, x, nblocks, stride, groups, ws=True):
    for b in range(nblocks):
        x = block(P, f"{name}.{b}.", x, stride if b == 0 else 1, groups, ws)
    return x


def upsample2x(x):
    """nn.Upsample(scale_factor=2, mode='trilinear') (align_corners=False), unet3D.py:1646."""
    return F.interpolate(x, scale_factor=2, mode="trilinear")


# ------------------------------------------------------------------------------------------------- A7
def trunk(P, x, layers=(1, 2, 2, 2, 2), groups=16, fusion_groups=16, ws=True, conv0=False):
    """Encoder/decoder trunk shared by unet3D_baseline.forward :663-711, unet3D.forward :1734-1784 and
    unet3D_g.forward :1568-1615. Returns (decoder output x1, bottleneck after fusionConv)."""
    if conv0:
        x = conv(x, P["conv0.weight"], 2, ws=ws)
    x = conv(x, P["conv1.weight"], 1, ws=ws)
    skips = []
    for i, name in enumerate(["layer0", "layer1", "layer2", "layer3", "layer4"]):
        x = layer(P, name, x, layers[i], 1 if i == 0 else 2, groups, ws)
        skips.append(x)
    x = conv(gn_relu(x, fusion_groups, P["fusionConv.0.weight"], P["fusionConv.0.bias"]), P["fusionConv.2.weight"], 1,
             ws=ws)
    bott = x
    for name, skip in zip(["x8_resb", "x4_resb", "x2_resb", "x1_resb"], [skips[3], skips[2], skips[1], skips[0]]):
        x = upsample2x(x) + skip
        x = layer(P, name, x, 1, 1, groups, ws)
    return x, bott


def precls(P, x, groups):
    """precls_conv = GN -> ReLU -> Conv3d 1^3 with bias, unet3D.py:629-633 / :1653-1657."""
    return F.conv3d(gn_relu(x, groups, P["precls_conv.0.weight"], P["precls_conv.0.bias"]),
                    P["precls_conv.2.weight"], P["precls_conv.2.bias"])


def baseline_forward(P, x, ws=True):
    """unet3D_baseline(layers=[1,2,2,2,2], num_classes, weight_std).forward, unet3D.py:663-718."""
    y, _ = trunk(P, x, ws=ws)
    return precls(P, y, 16)


def unet3d_g_forward(P, x, init_filter=8, layers=(1, 1, 1, 1, 1), ws=True):
    """unet3D_g.forward, unet3D.py:1568-1623: stride-2 conv0, GN(4) blocks, GN(init/2) fusion, GN(init/4) precls,
    final x2 trilinear upsample of the logits."""
    y, _ = trunk(P, x, layers=layers, groups=4, fusion_groups=init_filter // 2, ws=ws, conv0=True)
    return upsample2x(precls(P, y, init_filter // 4))


def unet3d_dyn_forward(P, x, task_id, ws=True):
    """UNet3D(num_classes, weight_std) = unet3D([1,2,2,2,2]) with the DynConv 8,8,2 head, unet3D.py:1734-1811."""
    y, bott = trunk(P, x, ws=ws)
    N = x.shape[0]
    onehot = F.one_hot(task_id.long(), 7).float().reshape(N, 7, 1, 1, 1)          # encoding_task :1688-1693
    feat = gn_relu(bott, 16, P["GAP.0.weight"], P["GAP.0.bias"]).mean(dim=(2, 3, 4), keepdim=True)  # GAP :1659-1663
    params = F.conv3d(torch.cat([feat, onehot], 1), P["controller.weight"], P["controller.bias"]).reshape(N, -1)
    head = precls(P, y, 16)                                                           # N x 8 x D x H x W
    D, H, W = head.shape[2:]
    h = head.reshape(1, -1, D, H, W)
    wn, bn = [64, 64, 16], [8, 8, 2]                                                  # :1790-1798
    splits = list(torch.split_with_sizes(params, wn + bn, dim=1))                    # parse_dynamic_params :1695-1718
    ws_, bs_ = splits[:3], splits[3:]
    for l in range(3):
        co = 8 if l < 2 else 2
        h = F.conv3d(h, ws_[l].reshape(N * co, -1, 1, 1, 1), bs_[l].reshape(N * co), groups=N)  # heads_forward :1720
        if l < 2:
            h = F.relu(h)
    return h.reshape(-1, 2, D, H, W)


# ------------------------------------------------------------------------------------------- A10 / A11
def edice_partial(inputs, target, mask=None, soft_max=True, uce=True):
    """EDiceLoss_partial.forward, loss_partial.py:71-99 with DiceLoss :10-57.

    Quirks kept: only ``mask[0]`` weights the whole batch; dice summed over all samples+voxels per class;
    loss divided by C (not sum of weights); BCE = torch BCELoss (mean over S*V, log clamped at -100)."""
    C = inputs.shape[1]
    p = torch.softmax(inputs, 1) if soft_max else torch.sigmoid(inputs)
    if mask is None:
        mask = [torch.ones(C) for _ in range(inputs.shape[0])]
    w = mask[0]
    loss = 0.0
    for i in range(C):
        t = (target == i).float()
        s = p[:, i]
        inter = torch.sum(s * t)
        y_sum = torch.sum(t * t)
        z_sum = torch.sum(s * s)
        d = 1 - (2 * inter + 1e-5) / (z_sum + y_sum + 1e-5)
        loss = loss + d * w[i]
    loss = loss / C
    if uce:
        ce = 0.0
        for l in range(C):
            ce = ce + F.binary_cross_entropy(p[:, l].float(), (target == l).float()) * w[l]
        loss = loss + ce
    return loss


# ------------------------------------------------------------------------------------------------- A14
def _soft_dice(p, t):
    """DiceLoss._dice_loss, loss_partial.py:24-36, mask all ones: 1 - (2 sum pt + 1e-5) / (sum p^2 + sum t^2 + 1e-5)."""
    return 1 - (2 * torch.sum(p * t) + 1e-5) / (torch.sum(p * p) + torch.sum(t * t) + 1e-5)


def edice_full(inputs, target, logits="softmax", uce=True):
    """EDiceLoss_full.forward, loss_partial.py:119-135 (DiceLoss over all C classes, weights 1, / C) + the
    cross entropy of the logits (nn.CrossEntropyLoss, mean) when uce."""
    C = inputs.shape[1]
    p = torch.softmax(inputs, 1) if logits == "softmax" else torch.sigmoid(inputs)
    t = target.long()
    dice = sum(_soft_dice(p[:, i], (t == i).float()) for i in range(C)) / C
    if uce:
        dice = dice + F.cross_entropy(inputs.float(), t)
    return dice


def get_loss_refine(output, label, dlist, aug_mask=1):
    """losses.py:46-62: sum over samples of EDiceLoss_full(2)(output[i:i+1], label == l+1, uce=False)."""
    loss = 0.
    for kk in range(aug_mask if aug_mask > 1 else 1):
        start = kk * len(dlist)
        for idx, l in enumerate(dlist):
            loss = loss + edice_full(output[start + idx:start + idx + 1], (label == (l + 1)).squeeze(1), uce=False)
    return loss


def partial_target(labels, sup_mask):
    """train_amos_atlas_final.py:252-255 (numpy): for l in 1..13, if not mask[l]: cmask[cmask == l] = 0."""
    cm = np.array(labels, dtype=np.float32, copy=True)
    for l in range(1, 14):
        if not sup_mask[l]:
            cm[cm == l] = 0
    return cm


def get_dice(preds, labels, num_class=13):
    """evaluate_amos.py:92-154 (atlas=None branch): argmax of softmax; per class l=1..num_class per-sample
    dice 2*sum(P*T)/(sum P + sum T + 1), sensitivity sum(P*T)/(sum T + 1), precision sum(P*T)/(sum P + 1),
    each averaged over samples. Returns three float64 numpy arrays."""
    am = torch.argmax(torch.softmax(preds, 1), 1)
    S = preds.shape[0]
    dices, senc, spec = [], [], []
    for l in range(1, num_class + 1):
        P = (am == l).reshape(S, -1).double()
        T = (labels == l).reshape(S, -1).double()
        num = (P * T).sum(1)
        dices.append((2 * num / (P.sum(1) + T.sum(1) + 1)).mean().item())
        senc.append((num / (T.sum(1) + 1)).mean().item())
        spec.append((num / (P.sum(1) + 1)).mean().item())
    return np.array(dices), np.array(senc), np.array(spec)


def get_dice2(preds, labels, num_class=13):
    """evaluate_amos.py:156-182 (atlas=None): organ l's prediction argmax(softmax(preds[l])) == 1 against
    labels == l+1, per organ dice 2PT/(P+T+1), sensitivity PT/(T+1), precision PT/(P+1)."""
    am = torch.argmax(torch.softmax(preds, 1), 1)
    d, se, sp = [], [], []
    for l in range(num_class):
        P = (am[l:l + 1] == 1).reshape(1, -1).double()
        T = (labels == l + 1).reshape(1, -1).double()
        num = (P * T).sum(1)
        d.append((2 * num / (P.sum(1) + T.sum(1) + 1)).mean().item())
        se.append((num / (T.sum(1) + 1)).mean().item())
        sp.append((num / (P.sum(1) + 1)).mean().item())
    return np.array(d), np.array(se), np.array(sp), am


# ---------------------------------------------------------------------------------------------- next f1
def gaussian_map(patch_size, sigma_scale=1.0 / 8):
    """_get_gaussian, evaluate_amos.py:184-197: scipy gaussian_filter (truncate 4.0, mode constant) of a centred
    delta = separable product of normalised 1-D kernels; scaled to max 1; zeros replaced by the min non-zero."""
    axes = []
    for n in patch_size:
        sigma = n * sigma_scale
        radius = int(4.0 * sigma + 0.5)
        xs = np.arange(-radius, radius + 1, dtype=np.float64)
        k = np.exp(-0.5 * (xs / sigma) ** 2)
        k /= k.sum()
        c = n // 2
        prof = np.zeros(n)
        for i in range(n):
            d = i - c
            if -radius <= d <= radius:
                prof[i] = k[d + radius]
        axes.append(prof)
    g = axes[0][:, None, None] * axes[1][None, :, None] * axes[2][None, None, :]
    g = g / g.max()
    g = g.astype(np.float32)
    g[g == 0] = g[g != 0].min()
    return g


def predict_sliding(pred_fn, image, tile_size, classes, tta=False):
    """predict_sliding, evaluate_amos.py:198-279, in float64 numpy. ``pred_fn(tile) -> [N, classes, td, th, tw]``
    stands for multi_net (:207-217: the mean over the nets, computed by the caller). Tiling, clamping, the flip
    TTA average, the Gaussian weighting of each tile and full /= count follow the reference line by line."""
    g = gaussian_map(tile_size)
    N, _, D, H, W = image.shape
    overlap = 1 / 4
    sHW = math.ceil(tile_size[1] * (1 - overlap))
    sD = math.ceil(tile_size[0] * (1 - overlap))
    nd = int(math.ceil((D - tile_size[0]) / sD) + 1)
    nr = int(math.ceil((H - tile_size[1]) / sHW) + 1)
    nc = int(math.ceil((W - tile_size[2]) / sHW) + 1)
    full = np.zeros((N, classes, D, H, W))
    count = np.zeros((N, classes, D, H, W))
    flips = [()] + ([(2,), (3,), (4,), (2, 3), (2, 4), (3, 4), (2, 3, 4)] if tta else [])
    for dep in range(nd):
        for row in range(nr):
            for col in range(nc):
                d1, x1, y1 = int(dep * sD), int(col * sHW), int(row * sHW)
                d2, x2, y2 = min(d1 + tile_size[0], D), min(x1 + tile_size[2], W), min(y1 + tile_size[1], H)
                d1, x1, y1 = max(d2 - tile_size[0], 0), max(x2 - tile_size[2], 0), max(y2 - tile_size[1], 0)
                img = image[:, :, d1:d2, y1:y2, x1:x2]
                pred = sum(np.flip(pred_fn(np.ascontiguousarray(np.flip(img, f))), f) if f else pred_fn(img)
                           for f in flips) / len(flips)
                count[:, :, d1:d2, y1:y2, x1:x2] += g
                full[:, :, d1:d2, y1:y2, x1:x2] += pred * g
    return full / count


# ---------------------------------------------------------------------------------------------- next f2
def eam_attn(P, pre, x, token, num_heads=4):
    """EAM.forward, unet3D.py:186-212, up to the returned ``attn`` (q k^T before the scaled softmax) — the only
    output unet3D_with_feam3 uses (its ``cm`` is discarded, :1134). x [B, N, C], token [1, Nt, C]. The kv / q
    reshapes use the TOKEN's batch (:189, :198), so B > 1 raises exactly as in the reference."""
    B, N, C = x.shape
    Bt, Nt, _ = token.shape
    xn = F.layer_norm(x, (C,), P[pre + "norm2.weight"], P[pre + "norm2.bias"], 1e-5)
    tn = F.layer_norm(token, (C,), P[pre + "norm3.weight"], P[pre + "norm3.bias"], 1e-5)
    kv = F.linear(xn, P[pre + "kv.weight"]).reshape(Bt, N, 2, num_heads, C // num_heads).permute(2, 0, 3, 1, 4)
    q = F.linear(tn, P[pre + "q.weight"]).reshape(Bt, Nt, num_heads, C // num_heads).permute(0, 2, 1, 3)
    return q @ kv[0].transpose(-2, -1)


def feam3_forward(P, tokens, x, num_classes, deep_up=False, use_cm=(True, True, True), training=True):
    """unet3D_with_feam3.forward, unet3D.py:1095-1190 (layers [1,2,2,2,2], GN 16): trunk + deep-supervision heads
    deepout1-3 (GN, ReLU, 1^3 conv + bias, :969-993) + EAM attention maps against the detached class tokens
    (:1131-1175; x8/x4/x2 upsampled to full size when deep_up) + detached feature copies. ``tokens`` =
    [class_token1 (nc-1 x 128), class_token2 (x 64), class_token3 (x 32)]."""
    x = conv(x, P["conv1.weight"], 1)
    skips = []
    for i, name in enumerate(["layer0", "layer1", "layer2", "layer3", "layer4"]):
        x = layer(P, name, x, (1, 2, 2, 2, 2)[i], 1 if i == 0 else 2, 16)
        skips.append(x)
    x = conv(gn_relu(x, 16, P["fusionConv.0.weight"], P["fusionConv.0.bias"]), P["fusionConv.2.weight"], 1)
    atten, deep, feats = [], [], []
    scales = [8, 4, 2]
    for k, (name, skip, eam) in enumerate(zip(["x8_resb", "x4_resb", "x2_resb"], skips[3:0:-1],
                                               ["eam84", "eam42", "eam21"])):
        x = layer(P, name, upsample2x(x) + skip, 1, 1, 16)
        pre = f"deepout{k + 1}."
        deep.append(F.conv3d(gn_relu(x, 16, P[pre + "0.weight"], P[pre + "0.bias"]), P[pre + "2.weight"],
                             P[pre + "2.bias"]))
        feats.append(x.detach().clone())
        if use_cm[k]:
            B, C = x.shape[:2]
            xt = x.reshape(B, C, -1).permute(0, 2, 1)
            cattn = eam_attn(P, eam + ".", xt, tokens[k].reshape(1, num_classes - 1, C).detach())
            a = cattn.mean(1).reshape((B, num_classes - 1) + tuple(x.shape[2:]))
            atten.append(F.interpolate(a, scale_factor=scales[k], mode="trilinear") if deep_up else a)
    x = layer(P, "x1_resb", upsample2x(x) + skips[0], 1, 1, 16)
    logits = precls(P, x, 16)
    return (logits, atten, deep, feats) if training else logits


def renew_token(tokens, features, mask, num_classes, alpha=0.01):
    """unet3D_with_feam3.renew_token, unet3D.py:1051-1068, in place on ``tokens``: for every class l with voxels
    in ``mask`` (== l+1), nearest-resized to each feature's size, token[l] <- (1-a) token[l] + a * mean. The mean
    is taken over ``x[cmask].reshape(C, -1)`` rows exactly as written (for B > 1 the rows are not channels)."""
    for index, x in enumerate(features):
        for l in range(num_classes):
            if (mask == (l + 1)).sum() != 0:
                cmask = F.interpolate((mask == (l + 1)).float(), x.shape[2:], mode="nearest").bool()
                cmask = cmask.repeat(1, x.shape[1], 1, 1, 1)
                if cmask.sum() == 0:
                    continue
                m = x[:, :][cmask].reshape(x.shape[1], -1).mean(-1).detach()
                tokens[index][l] = tokens[index][l] * (1 - alpha) + m * alpha
    return tokens


def state_shapes_feam3(num_classes=14):
    """Ordered (key, shape) list of the unet3D_with_feam3([1,2,2,2,2]) state_dict (registration order :949-1004)."""
    base = dict(state_shapes_baseline(num_classes))
    order = [k for k, _ in state_shapes_baseline(num_classes)]
    i8 = order.index("x8_resb.0.gn1.weight")
    head = [(k, base[k]) for k in order[:i8]]

    def blk(name):
        return [(k, base[k]) for k in order if k.startswith(name + ".")]

    def extra(k, c):
        e = [(f"deepout{k}.0.weight", (c,)), (f"deepout{k}.0.bias", (c,)),
             (f"deepout{k}.2.weight", (num_classes, c, 1, 1, 1)), (f"deepout{k}.2.bias", (num_classes,))]
        pre = {1: "eam84", 2: "eam42", 3: "eam21"}[k] + "."
        e += [(pre + "kv.weight", (2 * c, c)), (pre + "q.weight", (c, c)), (pre + "proj.weight", (c, c)),
              (pre + "proj.bias", (c,)), (pre + "norm2.weight", (c,)), (pre + "norm2.bias", (c,)),
              (pre + "norm3.weight", (c,)), (pre + "norm3.bias", (c,))]
        return e

    out = head + blk("x8_resb") + extra(1, 128) + blk("x4_resb") + extra(2, 64) + blk("x2_resb") + extra(3, 32)
    out += blk("x1_resb") + blk("precls_conv")
    return out


def _dice_loss_masked(score, target, mask):
    """DiceLoss._dice_loss, loss_partial.py:24-36: score[mask], target[mask.squeeze(1)], smooth 1e-5."""
    s = score[mask.bool()]
    t = target.float()[mask.squeeze(1).bool()]
    return 1 - (2 * torch.sum(s * t) + 1e-5) / (torch.sum(s * s) + torch.sum(t * t) + 1e-5)


def edice_full2(inputs, target, uce=True, mask=None, sigmoid=True):
    """EDiceLoss_full2.forward, loss_partial.py:150-170: masked soft dice of sigmoid(inputs) (or inputs) vs the
    soft target; + BCEWithLogits(inputs.squeeze(0), target) (mean, unmasked) when uce."""
    s = torch.sigmoid(inputs) if sigmoid else inputs
    if mask is None:
        mask = torch.ones_like(target).unsqueeze(0)
    d = _dice_loss_masked(s, target, mask)
    if uce:
        d = d + F.binary_cross_entropy_with_logits(inputs.float().squeeze(0), target.float())
    return d


def get_loss_consistency(output, target, mask, attns, refine_output, label_t, confi_=0.10, aux_weight=1,
                         weight_feature=0.1):
    """get_loss, losses.py:107-113 + 131-178 (refine_output given, no deep_out): EDiceLoss_partial(output) +
    sum over maps (3 attention maps, then softmax(output)[:, 1:]) and unsupervised organs gan (label_t[gan] == 0)
    of EDiceLoss_full2(map[:, gan], softmax(refine)[gan, 1], mask = refiner confident (p > 1-confi or p < confi),
    sigmoid except for the softmax map) / (num_classes - supcount) * [0.125, .25, .5, 1][idx] * weight_feature.
    ``refine_label`` (:134-157) is built by the reference but never read, so it is not restated."""
    dice_loss = edice_partial(output, target.squeeze(1), mask=mask)
    num_classes = output.shape[1] - 1
    weights = [0.125, 0.25, 0.5, 1]
    p = torch.softmax(refine_output, 1)
    confi = torch.logical_or(p > (1 - confi_), p < confi_).float()
    supcount = int(sum(1 for l in range(refine_output.shape[0]) if label_t[l]))
    maps = list(attns) + [torch.softmax(output, 1)[:, 1:]]
    aux = 0.0
    for idx, l in enumerate(maps):
        for gan in range(num_classes):
            if not label_t[gan]:
                cd = edice_full2(l[:, gan:gan + 1], p[gan:gan + 1, 1], uce=False, sigmoid=idx != 3,
                                 mask=confi[gan:gan + 1, 1:])
                aux = aux + cd / (num_classes - supcount) * weights[idx] * weight_feature
    return dice_loss + aux * aux_weight


# ---------------------------------------------------------------------------------------------- next f4
def truncate(ct, name):
    """AMOSDataSet_newatlas.truncate, MOTSDataset.py:171-186: CT (case id < 500) clipped to [-325, 325] and / 325;
    MRI z-scored with np.mean / np.std (population) of the whole (padded) array. numpy's own dtype rules, as the
    reference computes (an int16 CT array is clipped in place and divided in float64; a float32 MRI array is z-scored
    in float32 with numpy's pairwise sums): pinned bit-exact by G15."""
    ct = np.array(ct, copy=True)
    if float(name) < 500:
        ct[ct <= -325] = -325
        ct[ct >= 325] = 325
        return (ct - 0) / 325.
    ct = ct - np.mean(ct)
    return ct / np.std(ct)


def pad_image(img, target, lead=0):
    """pad_image / pad_image2, MOTSDataset.py:269-297: zero-pad the trailing three dims up to target."""
    pads = [(0, 0)] * lead + [(0, max(0, int(math.ceil(t - n)))) for t, n in zip(target, img.shape[lead:])]
    return np.pad(img, pads, "constant")


def get_item_tensors(image, label, catlas, name, crop_size, rng, usage="train"):
    """The tensor part of AMOSDataSet_newatlas.__getitem__ (MOTSDataset.py:355-384) after the file reads and the
    atlas resize: pad to crop + 5, truncate, random crop (rng.randint in the order b, c, a), (H, W, D) -> (D, H, W)."""
    cd, ch, cw = crop_size
    tgt = [ch + 5, cw + 5, cd + 5]
    image, label = pad_image(image, tgt), pad_image(label, tgt)
    catlas = pad_image(catlas, tgt, lead=1)
    image = truncate(image, name)
    if usage == "train":
        b = rng.randint(label.shape[0] - ch)
        c = rng.randint(label.shape[1] - cw)
        a = rng.randint(label.shape[2] - cd)
        image = image[b:b + ch, c:c + cw, a:a + cd]
        label = label[b:b + ch, c:c + cw, a:a + cd]
        catlas = catlas[:, b:b + ch, c:c + cw, a:a + cd]
    image = image[np.newaxis].transpose((0, 3, 1, 2)).astype(np.float32)
    label = label[np.newaxis].transpose((0, 3, 1, 2)).astype(np.float32)
    catlas = catlas.transpose((0, 3, 1, 2))
    return image, label, catlas


def aug_blur(x, sigma):
    """batchgenerators augment_gaussian_blur on one channel: scipy.ndimage.gaussian_filter(x, sigma, order=0)."""
    from scipy.ndimage import gaussian_filter
    return gaussian_filter(np.asarray(x, dtype=np.float64), sigma, order=0).astype(np.float32)


def aug_contrast(x, factor, preserve_range=True):
    """batchgenerators augment_contrast on one channel: (x - mean) * factor + mean, clipped to the original range."""
    x = np.asarray(x, dtype=np.float64)
    mn, lo, hi = x.mean(), x.min(), x.max()
    y = (x - mn) * factor + mn
    if preserve_range:
        y = np.clip(y, lo, hi)
    return y.astype(np.float32)


def params_from_module_dict(sd):
    return {k: v.detach().float().cpu() for k, v in sd.items()}


def state_shapes_baseline(num_classes=16, in_channel=1, init_filter=32, layers=(1, 2, 2, 2, 2), groups_ds=True,
                          conv0=False, dyn=False):
    """Ordered (key, shape) list of the reference state_dict for unet3D_baseline / unet3D / unet3D_g."""
    f = init_filter
    out = []
    if conv0:
        out.append(("conv0.weight", (f, in_channel, 3, 3, 3)))
        out.append(("conv1.weight", (f, f, 3, 3, 3)))
    else:
        out.append(("conv1.weight", (f, in_channel, 3, 3, 3)))

    def blk(pre, cin, cout, ds):
        o = [(pre + "gn1.weight", (cin,)), (pre + "gn1.bias", (cin,)), (pre + "conv1.weight", (cout, cin, 3, 3, 3)),
             (pre + "gn2.weight", (cout,)), (pre + "gn2.bias", (cout,)), (pre + "conv2.weight", (cout, cout, 3, 3, 3))]
        if ds:
            o += [(pre + "downsample.0.weight", (cin,)), (pre + "downsample.0.bias", (cin,)),
                  (pre + "downsample.2.weight", (cout, cin, 1, 1, 1))]
        return o

    chans = [(f, f), (f, 2 * f), (2 * f, 4 * f), (4 * f, 8 * f), (8 * f, 8 * f)]
    for i, (ci, co) in enumerate(chans):
        for b in range(layers[i]):
            cin = ci if b == 0 else co
            out += blk(f"layer{i}.{b}.", cin, co, b == 0 and (i > 0 or ci != co))
    out += [("fusionConv.0.weight", (8 * f,)), ("fusionConv.0.bias", (8 * f,)),
            ("fusionConv.2.weight", (8 * f, 8 * f, 1, 1, 1))]
    for name, ci, co in [("x8_resb", 8 * f, 4 * f), ("x4_resb", 4 * f, 2 * f), ("x2_resb", 2 * f, f), ("x1_resb", f, f)]:
        out += blk(f"{name}.0.", ci, co, ci != co)
    ncls = 8 if dyn else num_classes
    out += [("precls_conv.0.weight", (f,)), ("precls_conv.0.bias", (f,)),
            ("precls_conv.2.weight", (ncls, f, 1, 1, 1)), ("precls_conv.2.bias", (ncls,))]
    if dyn:
        out += [("GAP.0.weight", (256,)), ("GAP.0.bias", (256,)), ("controller.weight", (162, 263, 1, 1, 1)),
                ("controller.bias", (162,))]
    return out
