"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE in this container.

TEST INFRASTRUCTURE. Run here only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Everything it writes is data (inputs + expected outputs) in small .npz files; weights are not stored,
only the seed of oracle/weights_recipe.py. The reference is imported read-only from /root/reference with
the shims SURVEY.md §8c lists (no source of it is copied anywhere):
  * ``unet3D.unet3D.encoding_task``: the original moves the one-hot to ``.cuda()`` (unet3D.py:1688-1693);
    the shim builds the identical one-hot on the CPU.
  * ``loss_partial.autocast``: imported name is commented out (loss_partial.py:4, used :90); fp32 CPU
    ``autocast(enabled=False)`` is a no-op, so a nullcontext is semantically identical.
  * empty stub modules for ``cv2``, ``tensorboardX``, ``SimpleITK``, ``nibabel`` (not installed, unused by
    the functions exercised).
"""
import contextlib
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "oracle"))
from weights_recipe import apply_recipe, input_volume, label_volume  # noqa: E402

for name in ("cv2", "tensorboardX", "SimpleITK", "nibabel"):
    m = types.ModuleType(name)
    if name == "tensorboardX":
        m.SummaryWriter = object
    sys.modules.setdefault(name, m)
sys.path.insert(0, REF)

import unet3D as R  # noqa: E402
from loss_functions import loss_partial as RLP  # noqa: E402
import evaluate_amos as REV  # noqa: E402

R.unet3D.encoding_task = lambda self, t: F.one_hot(t.long(), 7).float()
RLP.autocast = lambda enabled=False: contextlib.nullcontext()

torch.set_num_threads(8)
torch.manual_seed(0)
OUT = HERE
SAMPLE_N = 4096


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {name}: {os.path.getsize(path) / 1024:.1f} KiB")


def grad_summary(model, n_sample=16):
    """Per-parameter grad L2 norm + grads at recipe-seeded flat indices (key order = state_dict)."""
    names, norms, idx_all, val_all = [], [], [], []
    for i, (k, p) in enumerate(model.named_parameters()):
        g = p.grad.detach().reshape(-1).double()
        rng = np.random.default_rng([1234, i])
        idx = rng.integers(0, g.numel(), size=n_sample)
        names.append(k)
        norms.append(g.norm().item())
        idx_all.append(idx)
        val_all.append(g[torch.from_numpy(idx)].numpy())
    return np.array(names), np.array(norms), np.stack(idx_all), np.stack(val_all)


def dice_arrays(preds, labels, num_class):
    dices, senc, spec, am = REV.get_dice(preds, labels, 1, num_class=num_class)
    return (np.array([float(d) for d in dices]), np.array([float(s) for s in senc]),
            np.array([float(s) for s in spec]))


def g1():
    m = R.UNet3D(num_classes=2, weight_std=True)
    apply_recipe(m, seed=0)
    m.eval()
    x = torch.from_numpy(input_volume((1, 1, 32, 32, 32), seed=1))
    task = torch.tensor([0])
    with torch.no_grad():
        logits = m(x, task)
    lab = torch.from_numpy(label_volume((1, 1, 32, 32, 32), 2, seed=2))
    d, se, sp = dice_arrays(logits, lab, 1)
    # backward through the dynamic head with a fixed upstream gradient
    m.train()
    x2 = torch.from_numpy(input_volume((2, 1, 32, 32, 32), seed=3))
    task2 = torch.tensor([0, 5])
    out = m(x2, task2)
    up = torch.from_numpy(input_volume(tuple(out.shape), seed=4))
    (out * up).sum().backward()
    names, norms, gidx, gval = grad_summary(m)
    save("g1_unet3d_dyn_32.npz", x=x.numpy(), task_id=task.numpy(), logits=logits.numpy(), labels=lab.numpy(),
         dice=d, senc=se, spec=sp, x2=x2.numpy(), task_id2=task2.numpy(), logits2=out.detach().numpy(),
         up2=up.numpy(), gnames=names, gnorm=norms, gidx=gidx, gval=gval)


def g2():
    m = R.unet3D_g([1, 1, 1, 1, 1], num_classes=2, weight_std=True, init_filter=8, in_channel=1)
    apply_recipe(m, seed=0)
    m.eval()
    x = torch.from_numpy(input_volume((1, 1, 32, 32, 32), seed=5))
    with torch.no_grad():
        logits = m(x)
    lab = torch.from_numpy(label_volume((1, 1, 32, 32, 32), 2, seed=6))
    d, se, sp = dice_arrays(logits, lab, 1)
    # the refiner configuration of train_amos_atlas_final.py:120 (init_filter 24, 2 input channels)
    r = R.unet3D_g([1, 1, 1, 1, 1], num_classes=2, weight_std=True, init_filter=24, in_channel=2)
    apply_recipe(r, seed=0)
    r.train()
    xr = torch.from_numpy(input_volume((1, 2, 32, 32, 32), seed=7))
    outr = r(xr)
    up = torch.from_numpy(input_volume(tuple(outr.shape), seed=8))
    (outr * up).sum().backward()
    names, norms, gidx, gval = grad_summary(r)
    save("g2_unet3d_g_32.npz", x=x.numpy(), logits=logits.numpy(), labels=lab.numpy(), dice=d, senc=se, spec=sp,
         xr=xr.numpy(), logits_r=outr.detach().numpy(), up_r=up.numpy(), gnames=names, gnorm=norms,
         gidx=gidx, gval=gval)


def loss_cases(C, S, spatial, seed):
    rng = np.random.default_rng([seed, 99])
    m_a = (rng.random(C) < 0.6).astype(np.int64)
    m_a[1] = 1
    m_b = np.zeros(C, dtype=np.int64)
    m_c1 = (rng.random(C) < 0.5).astype(np.int64)
    return {"a": [torch.from_numpy(m_a)], "zero": [torch.from_numpy(m_b)],
            "persample": [torch.from_numpy(m_a), torch.from_numpy(m_c1)]}


def g3():
    C = 16
    m = R.unet3D_baseline([1, 2, 2, 2, 2], num_classes=C, weight_std=True)
    apply_recipe(m, seed=0)
    m.train()
    x = torch.from_numpy(input_volume((2, 1, 16, 16, 16), seed=9, kind="ct"))
    lab = torch.from_numpy(label_volume((2, 1, 16, 16, 16), C, seed=10))
    masks = loss_cases(C, 2, (16, 16, 16), seed=11)
    logits, _, _ = m(x)
    edice = RLP.EDiceLoss_partial(C)
    losses = {}
    for k, mk in masks.items():
        losses[k] = float(edice(logits.detach(), lab.squeeze(1), mask=mk, soft_max=True))
    lg = logits.detach().clone().requires_grad_(True)
    la = edice(lg, lab.squeeze(1), mask=masks["a"], soft_max=True)
    la.backward()
    dlogits = lg.grad.numpy()
    m.zero_grad()
    loss = edice(logits, lab.squeeze(1), mask=masks["a"], soft_max=True)
    loss.backward()
    names, norms, gidx, gval = grad_summary(m)
    save("g3_baseline16_16.npz", x=x.numpy(), labels=lab.numpy(), logits=logits.detach().numpy(),
         mask_a=masks["a"][0].numpy(), mask_zero=masks["zero"][0].numpy(), mask_ps1=masks["persample"][1].numpy(),
         loss_a=losses["a"], loss_zero=losses["zero"], loss_persample=losses["persample"], dlogits=dlogits,
         gnames=names, gnorm=norms, gidx=gidx, gval=gval)


def g3b():
    """2x1x32^3 baseline16 logits sampled at seeded voxels (full tensor would be 4 MB)."""
    C = 16
    m = R.unet3D_baseline([1, 2, 2, 2, 2], num_classes=C, weight_std=True)
    apply_recipe(m, seed=0)
    m.eval()
    x = torch.from_numpy(input_volume((2, 1, 32, 32, 32), seed=12, kind="ct"))
    with torch.no_grad():
        logits = m(x)
    flat = logits.permute(0, 2, 3, 4, 1).reshape(-1, C)
    rng = np.random.default_rng([13, 13])
    vidx = rng.integers(0, flat.shape[0], size=SAMPLE_N)
    lab = torch.from_numpy(label_volume((2, 1, 32, 32, 32), C, seed=14))
    d, se, sp = dice_arrays(logits, lab, C - 1)
    save("g3b_baseline16_32.npz", x=x.numpy(), vidx=vidx, logits_s=flat[torch.from_numpy(vidx)].numpy(),
         mean=logits.mean((0, 2, 3, 4)).numpy(), std=logits.std((0, 2, 3, 4)).numpy(),
         amin=logits.amin((0, 2, 3, 4)).numpy(), amax=logits.amax((0, 2, 3, 4)).numpy(),
         labels=lab.numpy(), dice=d, senc=se, spec=sp)


def g4():
    """Per-op known-answer vectors at small shapes."""
    out = {}
    torch.manual_seed(0)
    for tag, (cin, cout, k, s, sp) in {"c3s1": (32, 32, 3, 1, 8), "c3s2": (32, 64, 3, 2, 8), "c1s2": (32, 64, 1, 2, 8),
                                       "c3s1b": (64, 32, 3, 1, 6), "c1s1": (64, 32, 1, 1, 6)}.items():
        conv = R.conv3x3x3(cin, cout, kernel_size=(k, k, k), stride=(s, s, s), padding=k // 2, weight_std=True)
        apply_recipe(conv, seed=1)
        x = torch.from_numpy(input_volume((2, cin, sp, sp, sp), seed=20)).requires_grad_(True)
        y = conv(x)
        up = torch.from_numpy(input_volume(tuple(y.shape), seed=21))
        (y * up).sum().backward()
        out[f"{tag}_x"] = x.detach().numpy()
        out[f"{tag}_y"] = y.detach().numpy()
        out[f"{tag}_up"] = up.numpy()
        out[f"{tag}_dx"] = x.grad.numpy()
        out[f"{tag}_dw"] = conv.weight.grad.numpy()
        out[f"{tag}_w"] = conv.weight.detach().numpy()
    # GroupNorm(16, 32) + ReLU
    gn = torch.nn.GroupNorm(16, 32)
    apply_recipe(gn, seed=2)
    x = (torch.from_numpy(input_volume((2, 32, 6, 7, 8), seed=22)) * 3 + 1.5).requires_grad_(True)
    y = F.relu(gn(x))
    up = torch.from_numpy(input_volume(tuple(y.shape), seed=23))
    (y * up).sum().backward()
    out.update(gn_x=x.detach().numpy(), gn_y=y.detach().numpy(), gn_up=up.numpy(), gn_dx=x.grad.numpy(),
               gn_dgamma=gn.weight.grad.numpy(), gn_dbeta=gn.bias.grad.numpy(), gn_gamma=gn.weight.detach().numpy(),
               gn_beta=gn.bias.detach().numpy())
    # trilinear x2 (align_corners=False) on odd sizes
    upm = torch.nn.Upsample(scale_factor=2, mode="trilinear")
    x = torch.from_numpy(input_volume((2, 8, 5, 6, 7), seed=24)).requires_grad_(True)
    y = upm(x)
    up = torch.from_numpy(input_volume(tuple(y.shape), seed=25))
    (y * up).sum().backward()
    out.update(up_x=x.detach().numpy(), up_y=y.detach().numpy(), up_up=up.numpy(), up_dx=x.grad.numpy())
    # partial Dice + BCE, C = 14 and 16
    for C in (14, 16):
        lg = (torch.from_numpy(input_volume((2, C, 8, 8, 8), seed=30 + C)) * 2).requires_grad_(True)
        lab = torch.from_numpy(label_volume((2, 8, 8, 8), C, seed=31 + C))
        rng = np.random.default_rng([32, C])
        mk = (rng.random(15 if C == 14 else C) < 0.6).astype(np.int64)
        loss = RLP.EDiceLoss_partial(C)(lg, lab, mask=[torch.from_numpy(mk)], soft_max=True)
        loss.backward()
        d, se, sp = dice_arrays(lg.detach(), lab.unsqueeze(1), C - 1)
        out.update({f"loss{C}_logits": lg.detach().numpy(), f"loss{C}_labels": lab.numpy(), f"loss{C}_mask": mk,
                    f"loss{C}_value": float(loss), f"loss{C}_dlogits": lg.grad.numpy(),
                    f"loss{C}_dice": d, f"loss{C}_senc": se, f"loss{C}_spec": sp})
    # soft_max=False (sigmoid) and uce=False variants, C = 14
    lg = out["loss14_logits"]
    lab = torch.from_numpy(out["loss14_labels"])
    for tag, kw in {"sig": dict(soft_max=False), "nouce": dict(uce=False)}.items():
        t = torch.from_numpy(lg).clone().requires_grad_(True)
        loss = RLP.EDiceLoss_partial(14)(t, lab, mask=[torch.from_numpy(out["loss14_mask"])], **kw)
        loss.backward()
        out[f"loss14{tag}_value"] = float(loss)
        out[f"loss14{tag}_dlogits"] = t.grad.numpy()
    save("g4_ops.npz", **out)


def g5():
    """Full-size 96^3 single-sample forward: summary + sampled voxels."""
    C = 16
    m = R.unet3D_baseline([1, 2, 2, 2, 2], num_classes=C, weight_std=True)
    apply_recipe(m, seed=0)
    m.eval()
    x = torch.from_numpy(input_volume((1, 1, 96, 96, 96), seed=40, kind="ct"))
    with torch.no_grad():
        logits = m(x)
    flat = logits.permute(0, 2, 3, 4, 1).reshape(-1, C)
    rng = np.random.default_rng([41, 41])
    vidx = rng.integers(0, flat.shape[0], size=SAMPLE_N)
    save("g5_baseline16_96.npz", vidx=vidx, logits_s=flat[torch.from_numpy(vidx)].numpy(),
         mean=logits.mean((0, 2, 3, 4)).numpy(), std=logits.std((0, 2, 3, 4)).numpy(),
         amin=logits.amin((0, 2, 3, 4)).numpy(), amax=logits.amax((0, 2, 3, 4)).numpy())


def g7():
    """f3: EDiceLoss_full (loss_partial.py:102-135) and get_loss_refine (losses.py:46-62) values + dlogits."""
    from loss_functions import losses as RL
    rng = np.random.default_rng([7, 99])
    sp = (12, 10, 8)
    out = {}
    lab = torch.from_numpy(rng.integers(0, 14, (1, 1) + sp).astype(np.float32))
    for tag, n in (("a1", 3), ("a2", 6)):
        lg = torch.from_numpy((rng.standard_normal((n, 2) + sp) * 2).astype(np.float32)).requires_grad_(True)
        v = RL.get_loss_refine(lg, lab, [2, 5, 7], 1 if tag == "a1" else 2)
        v.backward()
        out[f"ref_{tag}_logits"], out[f"ref_{tag}_value"], out[f"ref_{tag}_dlogits"] = \
            lg.detach().numpy(), v.detach().numpy(), lg.grad.numpy()
    out["ref_labels"] = lab.numpy()
    for tag, C, lgt, uce in (("s2u", 2, "softmax", True), ("s2n", 2, "softmax", False), ("g2n", 2, "sigmoid", False),
                             ("s4u", 4, "softmax", True)):
        lg = torch.from_numpy((rng.standard_normal((2, C) + sp) * 2).astype(np.float32)).requires_grad_(True)
        t = torch.from_numpy(rng.integers(0, C, (2,) + sp).astype(np.int64))
        v = RLP.EDiceLoss_full(C)(lg, t, logits=lgt, uce=uce)
        v.backward()
        out[f"full_{tag}_logits"], out[f"full_{tag}_target"] = lg.detach().numpy(), t.numpy()
        out[f"full_{tag}_value"], out[f"full_{tag}_dlogits"] = v.detach().numpy(), lg.grad.numpy()
    save("g7_refine_losses.npz", **out)


def g6():
    """Gaussian importance map of predict_sliding (evaluate_amos.py:184-197) for the 64x192x192 tile."""
    g = REV._get_gaussian((64, 192, 192), sigma_scale=1.0 / 8)
    rng = np.random.default_rng([42, 42])
    pts = np.stack([rng.integers(0, s, size=SAMPLE_N) for s in g.shape], 1)
    save("g6_gaussian.npz", line_d=g[:, 96, 96], line_h=g[32, :, 96], line_w=g[32, 96, :], corner=g[0, 0, 0],
         gmin=g.min(), gmax=g.max(), pts=pts, vals=g[pts[:, 0], pts[:, 1], pts[:, 2]])


def g8():
    """f2: unet3D_with_feam3 (unet3D.py:938-1190) — train-mode outputs (logits, attention maps with and without
    deep_up, deep-supervision maps, stored features), parameter gradients of a seeded projection of every output,
    eval-mode logits, renew_token (B = 1) and the renew_token row quirk at B = 2 (use_cm off, :1064)."""
    from weights_recipe import param_array
    nc = 14
    out = {}
    x = torch.from_numpy(input_volume((1, 1, 32, 32, 32), seed=80, kind="normal"))
    for tag, deep_up in (("nd", False), ("du", True)):
        m = R.unet3D_with_feam3([1, 2, 2, 2, 2], num_classes=nc, weight_std=True, deep_up=deep_up)
        apply_recipe(m, seed=0)
        for k in (1, 2, 3):
            setattr(m, f"class_token{k}", torch.from_numpy(param_array(f"class_token{k}",
                                                                       getattr(m, f"class_token{k}").shape, 0)))
        m.train()
        logits, att, deep, feats = m(x)
        rng = np.random.default_rng([81, 1 if deep_up else 0])
        proj = [logits] + att + deep
        ups = [torch.from_numpy(rng.standard_normal(t.shape).astype(np.float32)) for t in proj]
        sum((t * u).sum() for t, u in zip(proj, ups)).backward()
        # the projections are regenerated by the tests from the same seed (not stored); full-size maps sampled
        if not deep_up:
            out[f"{tag}_logits"] = logits.detach().numpy()
            for i in range(3):
                out[f"{tag}_att{i}"], out[f"{tag}_deep{i}"] = att[i].detach().numpy(), deep[i].detach().numpy()
        else:
            for i in range(3):
                flat = att[i].detach().reshape(-1)
                idx = np.random.default_rng([84, i]).integers(0, flat.numel(), size=SAMPLE_N)
                out[f"{tag}_att{i}_idx"], out[f"{tag}_att{i}_val"] = idx, flat[torch.from_numpy(idx)].numpy()
                out[f"{tag}_att{i}_sum"] = att[i].detach().double().sum().numpy()
        names, norms, gidx, gval = [], [], [], []
        for i, (k, p) in enumerate(m.named_parameters()):
            names.append(k)
            if p.grad is None:                      # eamXX.proj.* : the EAM's x output is discarded (:1134)
                norms.append(-1.0)
                gidx.append(np.zeros(16, np.int64))
                gval.append(np.zeros(16))
                continue
            g = p.grad.detach().reshape(-1).double()
            idx = np.random.default_rng([1234, i]).integers(0, g.numel(), size=16)
            norms.append(g.norm().item())
            gidx.append(idx)
            gval.append(g[torch.from_numpy(idx)].numpy())
        out[f"{tag}_gnames"], out[f"{tag}_gnorm"] = np.array(names), np.array(norms)
        out[f"{tag}_gidx"], out[f"{tag}_gval"] = np.stack(gidx), np.stack(gval)
        if not deep_up:
            for i in range(3):
                out[f"feat{i}"] = feats[i].numpy()
            # renew_token with a label volume missing some classes (B = 1)
            lab = np.random.default_rng([82, 0]).integers(0, nc, size=(1, 1, 32, 32, 32))
            lab[np.isin(lab, [3, 7])] = 0
            lab[:, :, :16][lab[:, :, :16] == 5] = 0
            lab[lab == 9] = 0                            # class 9 only at odd (d, h, w): nearest resizing picks
            lab[:, :, 1::10, 1::6, 1::4] = 9             # even source indices, so it vanishes at every feature size
            fmask = torch.from_numpy(lab.astype(np.float32))
            m.renew_token(feats, fmask)
            out["renew_mask"] = lab.astype(np.float32)
            for k in (1, 2, 3):
                out[f"renew_tok{k}"] = getattr(m, f"class_token{k}").numpy()
            m.eval()
            with torch.no_grad():
                out["eval_minus_train"] = (m(x) - logits.detach()).abs().max().numpy()
    # the renew_token reshape quirk at B = 2 (rows of x[cmask].reshape(C, -1) are not channels)
    m = R.unet3D_with_feam3([1, 2, 2, 2, 2], num_classes=nc, weight_std=True)
    rng = np.random.default_rng([83, 0])
    feats = [torch.from_numpy(rng.standard_normal((2, c, s, s, s)).astype(np.float32))
             for c, s in ((128, 2), (64, 4), (32, 8))]
    lab = rng.integers(0, 5, size=(2, 1, 16, 16, 16)).astype(np.float32)
    lab[0][lab[0] == 2] = 0
    toks = [torch.from_numpy(param_array(f"class_token{k}", (nc - 1, c), 0)) for k, c in ((1, 128), (2, 64), (3, 32))]
    for k in (1, 2, 3):
        setattr(m, f"class_token{k}", toks[k - 1].clone())
    m.renew_token(feats, torch.from_numpy(lab))
    for i in range(3):
        out[f"q_feat{i}"] = feats[i].numpy()
        out[f"q_tok{i + 1}"] = getattr(m, f"class_token{i + 1}").numpy()
    out["q_mask"] = lab
    try:
        m(torch.zeros(2, 1, 16, 16, 16))
        out["b2_raises"] = np.array(0)
    except RuntimeError:
        out["b2_raises"] = np.array(1)
    save("g8_feam3_32.npz", **out)


def g9():
    """f2/f3: the consistency branch of get_loss (losses.py:107-113, 131-178: EDiceLoss_partial + masked
    EDiceLoss_full2 between each attention map / the output's softmax and the refiner's confident foreground) and
    EDiceLoss_full2 itself (loss_partial.py:137-170): values + gradients w.r.t. output and attention maps."""
    from loss_functions import losses as RL
    rng = np.random.default_rng([9, 9])
    sp = (12, 10, 8)
    out = {}
    C = 14
    for tag, lt in (("mix", [1, 0, 0, 1, 0, 1, 1, 0, 0, 0, 1, 0, 0]), ("none", [0] * 13), ("all", [1] * 13)):
        lg = torch.from_numpy((rng.standard_normal((1, C) + sp) * 2).astype(np.float32)).requires_grad_(True)
        lab = torch.from_numpy(rng.integers(0, C, (1, 1) + sp).astype(np.float32))
        mvec = torch.from_numpy(np.concatenate([[1], rng.integers(0, 2, 14)]).astype(np.int64))
        att = [torch.from_numpy((rng.standard_normal((1, C - 1) + sp) * 3).astype(np.float32)).requires_grad_(True)
               for _ in range(3)]
        ref = torch.from_numpy((rng.standard_normal((C - 1, 2) + sp) * 3).astype(np.float32))
        label_t = torch.tensor(lt).float()
        attl = list(att)
        v, conf = RL.get_loss(lg, 0, [], lab, [mvec], None, attl, ref, label_t, weight_feature=0.07)
        assert len(attl) == 3
        v.backward()
        out[f"{tag}_logits"], out[f"{tag}_labels"], out[f"{tag}_mask"] = lg.detach().numpy(), lab.numpy(), mvec.numpy()
        out[f"{tag}_refine"], out[f"{tag}_label_t"] = ref.numpy(), label_t.numpy()
        out[f"{tag}_value"], out[f"{tag}_dlogits"] = v.detach().numpy(), lg.grad.numpy()
        for i in range(3):
            gr = att[i].grad   # None when every organ is supervised (no aux term touches the maps)
            out[f"{tag}_att{i}"] = att[i].detach().numpy()
            out[f"{tag}_datt{i}"] = gr.numpy() if gr is not None else np.zeros(att[i].shape, np.float32)
    # EDiceLoss_full2 alone: sigmoid / identity, with and without mask, uce on/off
    x = torch.from_numpy((rng.standard_normal((1, 1) + sp) * 2).astype(np.float32))
    t = torch.from_numpy(rng.uniform(0, 1, (1,) + sp).astype(np.float32))
    m = torch.from_numpy((rng.uniform(0, 1, (1, 1) + sp) > 0.4).astype(np.float32))
    out["f2_x"], out["f2_t"], out["f2_m"] = x.numpy(), t.numpy(), m.numpy()
    for tag, kw in (("sig_m", dict(uce=False, mask=m)), ("sig_nom", dict(uce=False)),
                    ("id_m", dict(uce=False, mask=m, sigmoid=False)), ("sig_uce", dict(uce=True, mask=m))):
        xi = (torch.sigmoid(x) if tag.startswith("id") else x).clone().requires_grad_(True)
        v = RLP.EDiceLoss_full2(2)(xi, t, **kw)
        v.backward()
        out[f"f2_{tag}_in"], out[f"f2_{tag}_value"], out[f"f2_{tag}_grad"] = xi.detach().numpy(), \
            v.detach().numpy(), xi.grad.numpy()
    save("g9_consistency.npz", **out)


def g10():
    """unet3D_with_feam2 (unet3D.py:721-936, the model evaluate_amos.py:571 builds): state_dict order, eval logits,
    and the ema=True train forward with a mask (in-forward class-token updates before each level's attention)."""
    from weights_recipe import param_array
    nc = 14
    out = {}
    x = torch.from_numpy(input_volume((1, 1, 32, 32, 32), seed=80, kind="normal"))
    lab = np.random.default_rng([82, 0]).integers(0, nc, size=(1, 1, 32, 32, 32))
    lab[np.isin(lab, [3, 7])] = 0
    mask = torch.from_numpy(lab.astype(np.float32))
    for tag, ema in (("eval", False), ("ema", True)):
        m = R.unet3D_with_feam2([1, 2, 2, 2, 2], num_classes=nc, weight_std=True, ema=ema, deep_up=True)
        apply_recipe(m, seed=0)   # class tokens are parameters here: the recipe's 2-D class_token rule applies
        if tag == "eval":
            out["keys"] = np.array(list(m.state_dict().keys()))
            m.eval()
            with torch.no_grad():   # the logits never depend on the tokens: G8's (same weights, same input)
                g8 = np.load(os.path.join(OUT, "g8_feam3_32.npz"))["nd_logits"]
                out["eval_minus_g8"] = np.abs(m(x).numpy() - g8).max()
        else:
            m.train()
            logits, att, deep = m(x, mask)
            out["ema_minus_g8"] = np.abs(logits.detach().numpy() - g8).max()
            for i in range(3):
                flat = att[i].detach().reshape(-1)
                idx = np.random.default_rng([85, i]).integers(0, flat.numel(), size=SAMPLE_N)
                out[f"ema_att{i}_idx"], out[f"ema_att{i}_val"] = idx, flat[torch.from_numpy(idx)].numpy()
                out[f"ema_deep{i}"] = deep[i].detach().numpy()
                out[f"ema_tok{i + 1}"] = getattr(m, f"class_token{i + 1}").detach().numpy()
    # train mode without ema: the in-place token update on a leaf that requires grad raises
    m = R.unet3D_with_feam2([1, 2, 2, 2, 2], num_classes=nc, weight_std=True)
    try:
        m.train()(x, mask)
        out["noema_raises"] = np.array(0)
    except RuntimeError:
        out["noema_raises"] = np.array(1)
    out["mask"] = lab.astype(np.float32)
    save("g10_feam2_32.npz", **out)


def g11():
    """get_dice2 (evaluate_amos.py:156-182): the refiner's per-organ binary Dice / sensitivity / precision."""
    rng = np.random.default_rng([11, 11])
    sp = (12, 10, 8)
    ref = torch.from_numpy((rng.standard_normal((13, 2) + sp) * 2).astype(np.float32))
    ref[3, 1] = ref[3, 0]                        # exact ties: argmax takes class 0
    lab = torch.from_numpy(rng.integers(0, 14, (1, 1) + sp).astype(np.float32))
    d, se, spc, am = REV.get_dice2(ref, lab, 1, num_class=13)
    save("g11_dice2.npz", refine=ref.numpy(), labels=lab.numpy(), dice=np.array([float(v) for v in d]),
         senc=np.array([float(v) for v in se]), spec=np.array([float(v) for v in spc]), argmax=am.numpy())


def g12():
    """Driver helpers on the import line (train_amos_atlas_final.py:34-35): utils.mask_aug and the discriminator
    losses SmoothCrossEntropyLoss / bce_loss (values + gradients)."""
    import utils as RU
    from loss_functions import losses as RL
    rng = np.random.default_rng([12, 12])
    m = rng.standard_normal((3, 1, 2, 3, 4)).astype(np.float32)
    out = {"aug_in": m, "aug_out": RU.mask_aug(m, 2), "aug_out3": RU.mask_aug(m, 3)}
    x = torch.from_numpy(rng.standard_normal((5, 2)).astype(np.float32)).requires_grad_(True)
    t = torch.from_numpy(rng.integers(0, 2, 5).astype(np.int64))
    for tag, kw in (("plain", {}), ("smooth", dict(smoothing=0.2)), ("sum", dict(reduction="sum"))):
        x.grad = None
        v = RL.SmoothCrossEntropyLoss(**kw)(x, t)
        v.backward()
        out[f"sce_{tag}_value"], out[f"sce_{tag}_grad"] = v.detach().numpy(), x.grad.numpy().copy()
    out["sce_x"], out["sce_t"] = x.detach().numpy(), t.numpy()
    x.grad = None
    xb = x.detach().clone().requires_grad_(True)
    y_pred = xb * 1.0
    y_pred.get_device = lambda: "cpu"   # the reference moves the labels with .to(y_pred.get_device())
    out["bce1_value"] = RL.bce_loss(y_pred, 1).detach().numpy()
    save("g12_driver_helpers.npz", **out)


def g13():
    """predict_sliding (evaluate_amos.py:211-279) itself, run here on CPU: its only device call, the per-tile
    ``torch.from_numpy(img).cuda()`` (:242), is shimmed to the identity (Tensor.cuda -> self) for the call. The
    networks are deterministic stand-ins with the module call signature net(img, task_id): a 3^3 convolution with
    fixed asymmetric weights (so tile borders and the TTA flips change the result) plus a per-class bias and a
    tanh. Cases: one net without TTA on a ragged volume; two nets with the 8-flip TTA (multi_net's mean, :198-209);
    a volume of exactly one tile. The weights are stored with the outputs (float64 full_probs, as returned)."""
    rng = np.random.default_rng([13, 13])

    class StandIn(torch.nn.Module):
        def __init__(self, w, b):
            super().__init__()
            self.w = torch.nn.Parameter(torch.from_numpy(w))
            self.b = torch.nn.Parameter(torch.from_numpy(b))

        def forward(self, x, task_id):
            return torch.tanh(F.conv3d(x, self.w, padding=1) + self.b.view(1, -1, 1, 1, 1))

    out = {}
    cases = [("a", (14, 27, 29), (8, 16, 16), 1, False), ("b", (14, 27, 29), (8, 16, 16), 2, True),
             ("c", (8, 16, 16), (8, 16, 16), 2, True)]
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        for tag, vol, tile, nnets, tta in cases:
            C = 3
            ws = [(rng.standard_normal((C, 1, 3, 3, 3)) * 0.5).astype(np.float32) for _ in range(nnets)]
            bs = [(rng.standard_normal(C) * 0.2).astype(np.float32) for _ in range(nnets)]
            nets = [StandIn(w, b).eval() for w, b in zip(ws, bs)]
            img = rng.standard_normal((1, 1) + vol).astype(np.float32)
            with torch.no_grad():
                full = REV.predict_sliding(None, nets, img, tile, C, 0, tta=tta)
            out[f"{tag}_img"], out[f"{tag}_w"], out[f"{tag}_b"] = img, np.stack(ws), np.stack(bs)
            out[f"{tag}_tile"], out[f"{tag}_tta"] = np.array(tile), np.array(int(tta))
            out[f"{tag}_full"] = full.numpy()
    finally:
        torch.Tensor.cuda = cuda
    save("g13_predict_sliding.npz", **out)


def _driver_lines(first, last):
    """Source lines first..last (1-based, inclusive) of the reference driver, dedented: the driver is not importable
    here (batchgenerators / SimpleITK / torchvision absent), so its own lines are run instead of a restatement."""
    import textwrap
    with open(os.path.join(REF, "train_amos_atlas_final.py")) as f:
        lines = f.read().splitlines()[first - 1:last]
    return textwrap.dedent("\n".join(lines))


def g14():
    """A12: the partial-label target of the driver on the reference's own supervision table. Runs the driver's
    mask_dict construction (train_amos_atlas_final.py:177-183; the cluster path of :178 replaced by the local
    /root/reference/supervise_mask.csv) and its 13 masked writes (:252-255) on seeded synthetic labels 0..15, for
    EVERY row of the table (241 volumes: CT rows with one labelled organ, the 40 all-zero MRI rows). The batch holds
    two samples, as the driver masks the whole batch with the first volume's row."""
    import csv
    import re
    src_dict = _driver_lines(177, 183)
    src_mask = _driver_lines(252, 255)
    assert "mask_file = " in src_dict and "cmask[cmask == l] = 0" in src_mask, "driver lines moved"
    import tempfile
    with open(os.path.join(REF, "supervise_mask.csv")) as f:  # the driver eval()s each cell: plain int lists only
        rows = list(csv.reader(f))
    assert rows[0] == ["name", "mask"] and all(re.fullmatch(r"\[[0-9, ]*\]", m) for _, m in rows[1:])
    # the driver's loop has no header skip (eval("mask") of the header row fails), so the cluster file had none: the
    # local copy is handed over without its header line
    tmp = tempfile.NamedTemporaryFile("w", suffix=".csv", delete=False)
    csv.writer(tmp).writerows(rows[1:])
    tmp.close()
    src_dict = re.sub(r'mask_file = "[^"]*"', f"mask_file = {tmp.name!r}", src_dict)
    ns = {"csv": csv, "np": np, "torch": torch}
    exec(compile(src_dict, "train_amos_atlas_final.py:177-183", "exec"), ns)
    mask_dict = ns["mask_dict"]
    rng = np.random.default_rng([14, 14])
    labels = torch.from_numpy(rng.integers(0, 16, (2, 1, 6, 7, 5)).astype(np.float32))
    names = [n for n, _ in rows[1:]]
    outs, masks = [], []
    for name in names:
        ns_m = {"labels": labels, "mask_dict": mask_dict, "volumeName": name}
        exec(compile(src_mask, "train_amos_atlas_final.py:252-255", "exec"), ns_m)
        outs.append(ns_m["cmask"].numpy().astype(np.uint8))
        masks.append(mask_dict[name].numpy().astype(np.int8))
    save("g14_partial_target.npz", names=np.array(names), masks=np.stack(masks), labels=labels.numpy(),
         cmask=np.stack(outs))


def _ref_lines(fname, first, last):
    import textwrap
    with open(os.path.join(REF, fname)) as f:
        lines = f.read().splitlines()[first - 1:last]
    return textwrap.dedent("\n".join(lines))


def g15():
    """f4 (deterministic half): AMOSDataSet_newatlas.__getitem__'s tensor work run from the reference's own lines
    (MOTSDataset.py is not importable here: batchgenerators / SimpleITK absent). The methods ``truncate`` (:171-186),
    ``pad_image`` (:269-282), ``pad_image2`` (:284-297) are exec'd into a class body and the getitem lines :370-397
    (pad to crop + 5, truncate, random crop, transpose, astype) run on seeded synthetic volumes as sitk would return
    them ([H, W, D]; CT int16 HU, MRI float32 intensities) and a 13-channel atlas already resized to the image
    (:364). ``np.random`` is a seeded RandomState whose draws (b, c, a) are recorded; the device path draws from a
    RandomState with the same seed. Cases: CT and MRI, volumes smaller and larger than crop + 5, train and valid."""
    import math
    src_methods = "\n".join(_ref_lines("MOTSDataset.py", a, b) for a, b in ((171, 186), (269, 282), (284, 297)))
    src_get = _ref_lines("MOTSDataset.py", 370, 397).replace("return image.copy(), label.copy(), name, name, catlas",
                                                           "out = (image.copy(), label.copy(), catlas)")
    assert "def truncate(self, CT, task_id):" in src_methods and "def pad_image2" in src_methods
    assert "image = self.truncate(image, name)" in src_get and "out = (" in src_get, "reference lines moved"
    ns = {"np": np, "math": math}
    exec(compile("class DS:\n" + "\n".join("    " + ln for ln in src_methods.splitlines()),
                 "MOTSDataset.py:171-297", "exec"), ns)
    cases = [  # tag, name, shape [H, W, D], crop (d, h, w), usage, seed
        ("ct_small", "0007", (16, 30, 11), (8, 20, 16), "train", 151),
        ("ct_big", "0123", (30, 34, 20), (8, 16, 24), "train", 152),
        ("mri_small", "0541", (18, 20, 9), (8, 16, 16), "train", 153),
        ("mri_big", "0598", (28, 26, 22), (12, 16, 20), "train", 154),
        ("ct_valid", "0011", (14, 22, 12), (8, 16, 16), "valid", 155),
        ("mri_valid", "0512", (24, 15, 13), (8, 16, 16), "valid", 156),
    ]
    out = {}
    for tag, name, shp, crop, usage, seed in cases:
        g = np.random.default_rng([15, seed])
        if int(name) < 500:
            image = g.integers(-1100, 1400, shp).astype(np.int16)
        else:
            image = (g.gamma(2.0, 150.0, shp)).astype(np.float32)
        label = g.integers(0, 16, shp).astype(np.uint8)
        catlas = (g.integers(0, 65, (13,) + shp) / 64.0).astype(np.float32)  # atlas probabilities (compressible)
        ds = ns["DS"]()
        ds.crop_d, ds.crop_h, ds.crop_w = crop
        ds.usage = usage

        class _Rec:
            def __init__(self, seed):
                self.rs, self.draws = np.random.RandomState(seed), []

            def randint(self, *a):
                v = self.rs.randint(*a)
                self.draws.append(int(v))
                return v
        rec = _Rec(seed)
        npx = types.SimpleNamespace(**{k: getattr(np, k) for k in ("newaxis", "float32")})
        npx.random = rec
        env = {"self": ds, "image": image.copy(), "label": label.copy(), "catlas": catlas.copy(), "name": name,
               "np": npx}
        exec(compile(src_get, "MOTSDataset.py:370-397", "exec"), env)
        im, lb, ca = env["out"]
        for k, v in (("image_in", image), ("label_in", label), ("catlas_in", catlas), ("image", im), ("label", lb),
                     ("catlas", ca)):
            out[f"{tag}_{k}"] = v
        out[f"{tag}_name"], out[f"{tag}_crop"] = np.array(name), np.array(crop)
        out[f"{tag}_usage"], out[f"{tag}_seed"] = np.array(usage), np.array(seed)
        out[f"{tag}_draws"] = np.array(rec.draws, dtype=np.int64)
    save("g15_crop_patch.npz", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["g1", "g2", "g3", "g3b", "g4", "g5", "g6", "g7", "g8", "g9", "g10", "g11", "g12", "g13",
                             "g14", "g15"]
    for w in which:
        globals()[w]()
