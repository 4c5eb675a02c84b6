"""GPU parity of the native HIP path (through the C ABI) against the reference golden vectors and the CPU
oracle. fp32 mode is the parity mode (north_star: logits <= 1e-3 max-abs, Dice <= 1e-4); bf16 runs are
checked against the oracle on the same bf16-rounded operands with looser, stated tolerances."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref_cpu as O
from oracle.weights_recipe import apply_recipe, input_volume, label_volume, recipe_state_dict

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-3   # north_star: fp32 logits within 1e-3 max-abs of the reference CPU forward
DICE_TOL = 1e-4    # north_star: Dice within 1e-4


def _model(kind, **kw):
    import unet3D
    if kind == "baseline":
        m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=kw.get("C", 16), weight_std=True)
    elif kind == "g":
        m = unet3D.unet3D_g(kw.get("layers", [1] * 5), num_classes=2, weight_std=True,
                            init_filter=kw["f"], in_channel=kw["cin"])
    elif kind == "dyn":
        m = unet3D.UNet3D(num_classes=2, weight_std=True)
    apply_recipe(m, seed=0)
    return m


# Sampled gradient entries (gidx / gval: 16 recipe-seeded flat indices per parameter, tests/golden/gen_golden.py
# grad_summary). A tap-permuted or flipped weight gradient keeps the L2 norm but moves the entries by ~1.4x the
# parameter's gradient RMS; fp32 accumulation-order noise moves them by far less (entry-wise gradients of the
# shallow layers are ill-conditioned: ~1% of an entry for a 1e-7 forward perturbation), so the bound is
# stated against the RMS: max |g_i - ref_i| <= ENTRY_TOL x ||ref|| / sqrt(numel). Measured worst: G3 2.4e-5,
# G2 1.1e-5, G1 2.0e-2 (x2_resb.0.gn1.bias; the dynamic head's per-sample convs sit between the loss and the trunk).
ENTRY_TOL = 0.1


def _check_entries(P, g, tol=ENTRY_TOL):
    worst = (0.0, "")
    for i, k in enumerate(g["gnames"]):
        gr = P[str(k)].grad.reshape(-1).double().cpu()
        rms = float(g["gnorm"][i]) / np.sqrt(gr.numel())
        if rms == 0:
            continue
        got = gr[torch.from_numpy(g["gidx"][i])].numpy()
        e = float(np.abs(got - g["gval"][i]).max()) / rms
        worst = max(worst, (e, str(k)))
        assert e <= tol, f"{k}: sampled gradient entries off by {e:.3e} x RMS"
    print(f"worst sampled-entry error {worst[0]:.2e} x RMS ({worst[1]})")


# ------------------------------------------------------------------------------------------ per-op
@pytest.mark.parametrize("tag,s", [("c3s1", 1), ("c3s2", 2), ("c1s2", 2), ("c3s1b", 1), ("c1s1", 1)])
def test_ws_conv_fwd_bwd_vs_golden(gpu, tag, s):
    import unet3D
    g = golden("g4_ops.npz")
    w = torch.from_numpy(g[f"{tag}_w"])
    cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
    conv = unet3D.Conv3d(cin, cout, kernel_size=(k, k, k), stride=(s, s, s), padding=k // 2).to(gpu)
    with torch.no_grad():
        conv.weight.copy_(w.to(gpu))
    x = torch.from_numpy(g[f"{tag}_x"]).to(gpu).requires_grad_(True)
    y = conv(x)
    # fp32 MFMA (exact fp32 FMA chain) vs the CPU conv: summation order only -> 4e-6 of the output scale
    assert np.abs(y.detach().cpu().numpy() - g[f"{tag}_y"]).max() < 4e-6 * np.abs(g[f"{tag}_y"]).max()
    (y * torch.from_numpy(g[f"{tag}_up"]).to(gpu)).sum().backward()
    assert np.abs(x.grad.cpu().numpy() - g[f"{tag}_dx"]).max() < 4e-6 * np.abs(g[f"{tag}_dx"]).max()
    dw = conv.weight.grad.cpu().numpy()
    np.testing.assert_allclose(dw, g[f"{tag}_dw"], atol=2e-3 * np.abs(g[f"{tag}_dw"]).max(), rtol=1e-4)


def test_block_gn_fwd_bwd_vs_oracle(gpu):
    """NoBottleneck (GN prologue, residual epilogue, GN backward) on a 24^3 ragged-ish volume."""
    import unet3D
    torch.manual_seed(0)
    for cin, cout, s in [(32, 64, 2), (64, 64, 1), (64, 32, 1)]:
        ds = None
        if s != 1 or cin != cout:
            ds = torch.nn.Sequential(torch.nn.GroupNorm(16, cin), torch.nn.ReLU(True),
                                     unet3D.conv3x3x3(cin, cout, (1, 1, 1), (s, s, s), 0, weight_std=True))
        blk = unet3D.NoBottleneck(cin, cout, (s, s, s), downsample=ds, weight_std=True)
        apply_recipe(blk, seed=3)
        P = {k: v.detach().clone().requires_grad_(True) for k, v in blk.state_dict().items()}
        x = torch.from_numpy(input_volume((2, cin, 12, 10, 14), seed=5) * 2 + 0.5)
        xr = x.clone().requires_grad_(True)
        yr = O.block(P, "", xr, s, 16)
        up = torch.from_numpy(input_volume(tuple(yr.shape), seed=6))
        (yr * up).sum().backward()
        blk = blk.to(gpu)
        xg = x.to(gpu).requires_grad_(True)
        yg = blk(xg)
        assert (yg.detach().cpu() - yr.detach()).abs().max().item() < 4e-6 * yr.abs().max().item()
        (yg * up.to(gpu)).sum().backward()
        assert (xg.grad.cpu() - xr.grad).abs().max().item() < 1e-5 * xr.grad.abs().max().item()
        for k, p in blk.named_parameters():
            ref = P[k].grad
            err = (p.grad.cpu() - ref).norm().item() / max(ref.norm().item(), 1e-12)
            assert err < 1e-4, (k, err)


def test_upsample_fwd_bwd_vs_golden(gpu):
    from u3d import ops
    g = golden("g4_ops.npz")
    x = torch.from_numpy(g["up_x"]).to(gpu).permute(0, 2, 3, 4, 1).contiguous()
    y = ops.upsample2x_add(x)
    assert np.abs(y.permute(0, 4, 1, 2, 3).cpu().numpy() - g["up_y"]).max() < 1e-6
    dy = torch.from_numpy(g["up_up"]).to(gpu).permute(0, 2, 3, 4, 1).contiguous()
    dx = ops.upsample2x_bwd(dy, tuple(x.shape))
    assert np.abs(dx.permute(0, 4, 1, 2, 3).cpu().numpy() - g["up_dx"]).max() < 1e-5
    # odd channel count (logit upsample of unet3D_g, C=2) and a skip add
    x2 = torch.randn(1, 3, 4, 5, 2, device=gpu)
    sk = torch.randn(1, 6, 8, 10, 2, device=gpu)
    y2 = ops.upsample2x_add(x2, sk)
    ref = O.upsample2x(x2.permute(0, 4, 1, 2, 3).cpu()) + sk.permute(0, 4, 1, 2, 3).cpu()
    assert (y2.permute(0, 4, 1, 2, 3).cpu() - ref).abs().max().item() < 1e-6


@pytest.mark.parametrize("C", [14, 16])
def test_partial_loss_vs_golden(gpu, C):
    from loss_functions.loss_partial import EDiceLoss_partial
    g = golden("g4_ops.npz")
    lg = torch.from_numpy(g[f"loss{C}_logits"]).to(gpu).requires_grad_(True)
    lab = torch.from_numpy(g[f"loss{C}_labels"]).to(gpu)
    loss = EDiceLoss_partial(C)(lg, lab, mask=[torch.from_numpy(g[f"loss{C}_mask"])])
    np.testing.assert_allclose(loss.item(), float(g[f"loss{C}_value"]), rtol=2e-6, atol=1e-6)
    loss.backward()
    np.testing.assert_allclose(lg.grad.cpu().numpy(), g[f"loss{C}_dlogits"], rtol=1e-4,
                               atol=1e-6 * np.abs(g[f"loss{C}_dlogits"]).max())


@pytest.mark.parametrize("tag,kw", [("sig", dict(soft_max=False)), ("nouce", dict(uce=False))])
def test_partial_loss_variants(gpu, tag, kw):
    from loss_functions.loss_partial import EDiceLoss_partial
    g = golden("g4_ops.npz")
    lg = torch.from_numpy(g["loss14_logits"]).to(gpu).requires_grad_(True)
    loss = EDiceLoss_partial(14)(lg, torch.from_numpy(g["loss14_labels"]).to(gpu),
                                 mask=[torch.from_numpy(g["loss14_mask"])], **kw)
    np.testing.assert_allclose(loss.item(), float(g[f"loss14{tag}_value"]), rtol=2e-6, atol=1e-6)
    loss.backward()
    ref = g[f"loss14{tag}_dlogits"]
    np.testing.assert_allclose(lg.grad.cpu().numpy(), ref, rtol=1e-4, atol=1e-6 * np.abs(ref).max())


def test_partial_loss_zero_mask_and_short_mask(gpu):
    from loss_functions.loss_partial import EDiceLoss_partial
    lg = torch.randn(2, 16, 4, 4, 4, device=gpu, requires_grad=True)
    lab = torch.randint(0, 16, (2, 4, 4, 4), device=gpu).float()
    loss = EDiceLoss_partial(16)(lg, lab, mask=[torch.zeros(16, dtype=torch.int64)])
    assert loss.item() == 0.0
    loss.backward()
    assert lg.grad.abs().max().item() == 0.0
    with pytest.raises(IndexError):
        EDiceLoss_partial(16)(lg, lab, mask=[torch.ones(15, dtype=torch.int64)])


@pytest.mark.parametrize("C", [14, 16])
def test_dice_metric_vs_golden(gpu, C):
    from evaluate_amos import get_dice
    g = golden("g4_ops.npz")
    lg = torch.from_numpy(g[f"loss{C}_logits"]).to(gpu)
    lab = torch.from_numpy(g[f"loss{C}_labels"]).to(gpu).unsqueeze(1)
    d, se, sp, am = get_dice(lg, lab, 1, num_class=C - 1)
    np.testing.assert_allclose([float(v) for v in d], g[f"loss{C}_dice"], atol=DICE_TOL)
    np.testing.assert_allclose([float(v) for v in se], g[f"loss{C}_senc"], atol=DICE_TOL)
    np.testing.assert_allclose([float(v) for v in sp], g[f"loss{C}_spec"], atol=DICE_TOL)
    assert torch.equal(am.cpu(), torch.argmax(torch.softmax(lg.cpu(), 1), 1))


# ------------------------------------------------------------------------------------------ models
def test_g3_baseline16_forward_loss_backward(gpu):
    from loss_functions.loss_partial import EDiceLoss_partial
    g = golden("g3_baseline16_16.npz")
    m = _model("baseline").to(gpu).train()
    logits, a, b = m(torch.from_numpy(g["x"]).to(gpu))
    assert a == [] and b == []
    assert np.abs(logits.detach().cpu().numpy() - g["logits"]).max() < LOGIT_TOL
    lab = torch.from_numpy(g["labels"]).to(gpu).squeeze(1)
    ma = torch.from_numpy(g["mask_a"])
    crit = EDiceLoss_partial(16)
    for key, mask in [("loss_zero", [torch.from_numpy(g["mask_zero"])]),
                      ("loss_persample", [ma, torch.from_numpy(g["mask_ps1"])])]:
        np.testing.assert_allclose(crit(logits.detach(), lab, mask=mask).item(), float(g[key]), rtol=1e-4, atol=1e-6)
    loss = crit(logits, lab, mask=[ma])
    np.testing.assert_allclose(loss.item(), float(g["loss_a"]), rtol=1e-4, atol=1e-6)
    loss.backward()
    for i, k in enumerate(g["gnames"]):
        p = dict(m.named_parameters())[k]
        gr = p.grad.reshape(-1).double().cpu()
        np.testing.assert_allclose(gr.norm().item(), g["gnorm"][i], rtol=2e-3, atol=1e-9, err_msg=k)
    _check_entries(dict(m.named_parameters()), g)


def test_g3b_g5_sampled_logits_and_dice(gpu):
    for name, shape in [("g3b_baseline16_32.npz", None), ("g5_baseline16_96.npz", (1, 1, 96, 96, 96))]:
        g = golden(name)
        m = _model("baseline").to(gpu).eval()
        x = torch.from_numpy(g["x"] if shape is None else input_volume(shape, seed=40, kind="ct")).to(gpu)
        with torch.no_grad():
            y = m(x)
        flat = y.permute(0, 2, 3, 4, 1).reshape(-1, 16)[torch.from_numpy(g["vidx"]).to(gpu)].cpu().numpy()
        assert np.abs(flat - g["logits_s"]).max() < LOGIT_TOL, name
        np.testing.assert_allclose(y.mean((0, 2, 3, 4)).cpu().numpy(), g["mean"], atol=1e-4)
        np.testing.assert_allclose(y.amax((0, 2, 3, 4)).cpu().numpy(), g["amax"], atol=LOGIT_TOL)
        if "dice" in g:
            from evaluate_amos import get_dice
            d, _, _, _ = get_dice(y, torch.from_numpy(g["labels"]).to(gpu), 1, num_class=15)
            np.testing.assert_allclose([float(v) for v in d], g["dice"], atol=DICE_TOL)


def test_g2_unet3d_g_forward_and_refiner_backward(gpu):
    g = golden("g2_unet3d_g_32.npz")
    m = _model("g", f=8, cin=1).to(gpu).eval()
    with torch.no_grad():
        y = m(torch.from_numpy(g["x"]).to(gpu))
    assert np.abs(y.cpu().numpy() - g["logits"]).max() < LOGIT_TOL
    from evaluate_amos import get_dice
    d, _, _, _ = get_dice(y, torch.from_numpy(g["labels"]).to(gpu), 1, num_class=1)
    np.testing.assert_allclose([float(v) for v in d], g["dice"], atol=DICE_TOL)
    r = _model("g", f=24, cin=2).to(gpu).train()
    yr = r(torch.from_numpy(g["xr"]).to(gpu))
    assert np.abs(yr.detach().cpu().numpy() - g["logits_r"]).max() < LOGIT_TOL
    (yr * torch.from_numpy(g["up_r"]).to(gpu)).sum().backward()
    P = dict(r.named_parameters())
    for i, k in enumerate(g["gnames"]):
        np.testing.assert_allclose(P[k].grad.double().norm().item(), g["gnorm"][i], rtol=5e-3, err_msg=k)
    _check_entries(P, g)


def test_g1_unet3d_dynconv_forward_dice(gpu):
    g = golden("g1_unet3d_dyn_32.npz")
    m = _model("dyn").to(gpu).eval()
    with torch.no_grad():
        y = m(torch.from_numpy(g["x"]).to(gpu), torch.from_numpy(g["task_id"]))
        y2 = m(torch.from_numpy(g["x2"]).to(gpu), torch.from_numpy(g["task_id2"]))
    assert np.abs(y.cpu().numpy() - g["logits"]).max() < LOGIT_TOL
    assert np.abs(y2.cpu().numpy() - g["logits2"]).max() < LOGIT_TOL
    from evaluate_amos import get_dice
    d, se, sp, _ = get_dice(y, torch.from_numpy(g["labels"]).to(gpu), 1, num_class=1)
    np.testing.assert_allclose([float(v) for v in d], g["dice"], atol=DICE_TOL)


def test_g1_unet3d_dynconv_backward(gpu):
    """UNet3D DynConv 8,8,2 trained natively: every parameter gradient (trunk, precls, GAP GroupNorm, controller)
    against the reference's autograd on the same weights / input / upstream gradient (golden G1)."""
    g = golden("g1_unet3d_dyn_32.npz")
    m = _model("dyn").to(gpu).train()
    y = m(torch.from_numpy(g["x2"]).to(gpu), torch.from_numpy(g["task_id2"]))
    assert np.abs(y.detach().cpu().numpy() - g["logits2"]).max() < LOGIT_TOL
    (y * torch.from_numpy(g["up2"]).to(gpu)).sum().backward()
    P = dict(m.named_parameters())
    for i, k in enumerate(g["gnames"]):
        gr = P[k].grad.reshape(-1).double().cpu()
        np.testing.assert_allclose(gr.norm().item(), g["gnorm"][i], rtol=2e-3, atol=1e-9, err_msg=k)
    _check_entries(P, g)
    names = set(str(k) for k in g["gnames"])
    assert {"controller.weight", "controller.bias", "GAP.0.weight", "GAP.0.bias"} <= names


def test_bf16_mode_close_to_fp32(gpu):
    """bf16 activations/weights with fp32 accumulation: logits track the fp32 path (stated tolerance 0.25
    max-abs on O(1..10) logits after 36 bf16 layers), loss within 1e-2 relative."""
    from loss_functions.loss_partial import EDiceLoss_partial
    g = golden("g3b_baseline16_32.npz")
    m = _model("baseline").to(gpu).train()
    x = torch.from_numpy(g["x"]).to(gpu)
    lab = torch.from_numpy(g["labels"]).to(gpu).squeeze(1)
    y32, _, _ = m(x)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y16, _, _ = m(x)
    assert y16.dtype == torch.float32
    err = (y16 - y32).abs().max().item()
    assert err < 0.25 * max(1.0, y32.abs().max().item() / 10), err
    mk = [torch.ones(16, dtype=torch.int64)]
    l32 = EDiceLoss_partial(16)(y32, lab, mask=mk)
    l16 = EDiceLoss_partial(16)(y16, lab, mask=mk)
    assert abs(l16.item() - l32.item()) < 1e-2 * abs(l32.item())
    l16.backward()
    gn = m.layer0[0].conv1.weight.grad
    assert torch.isfinite(gn).all() and gn.abs().max() > 0


def test_cpu_tensor_raises(gpu):
    import unet3D
    from u3d import U3DError
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], 16, True)
    with pytest.raises(U3DError):
        m(torch.zeros(1, 1, 16, 16, 16))


# ------------------------------------------------------------------------------------ f3 refiner losses
def test_g7_get_loss_refine_and_edice_full(gpu):
    """loss_functions.losses.get_loss_refine / loss_partial.EDiceLoss_full (fused HIP loss, cross-entropy mode)
    against the reference's own values and dlogits (G7)."""
    from loss_functions import losses, loss_partial
    g = golden("g7_refine_losses.npz")
    lab = torch.from_numpy(g["ref_labels"]).to(gpu)
    for tag, aug in (("a1", 1), ("a2", 2)):
        lg = torch.from_numpy(g[f"ref_{tag}_logits"]).to(gpu).requires_grad_(True)
        v = losses.get_loss_refine(lg, lab, [2, 5, 7], aug)
        v.backward()
        np.testing.assert_allclose(float(v), float(g[f"ref_{tag}_value"]), rtol=1e-4)
        np.testing.assert_allclose(lg.grad.cpu().numpy(), g[f"ref_{tag}_dlogits"], rtol=1e-3, atol=1e-7)
    for tag, C, lgt, uce in (("s2u", 2, "softmax", True), ("s2n", 2, "softmax", False), ("g2n", 2, "sigmoid", False),
                             ("s4u", 4, "softmax", True)):
        lg = torch.from_numpy(g[f"full_{tag}_logits"]).to(gpu).requires_grad_(True)
        t = torch.from_numpy(g[f"full_{tag}_target"]).to(gpu)
        v = loss_partial.EDiceLoss_full(C)(lg, t, logits=lgt, uce=uce)
        v.backward()
        np.testing.assert_allclose(float(v), float(g[f"full_{tag}_value"]), rtol=1e-4)
        np.testing.assert_allclose(lg.grad.cpu().numpy(), g[f"full_{tag}_dlogits"], rtol=1e-3, atol=1e-7)


def test_partial_target_vs_oracle(gpu):
    """A12 (train_amos_atlas_final.py:252-255) as one device pass, batch mask and per-sample masks."""
    from loss_functions import losses
    from u3d import ops
    rng = np.random.default_rng(3)
    lab = rng.integers(0, 16, (2, 1, 9, 10, 11)).astype(np.float32)
    mask = rng.integers(0, 2, 15).astype(np.int64)
    got = losses.make_partial_target(torch.from_numpy(lab).to(gpu), torch.from_numpy(mask)).cpu().numpy()
    np.testing.assert_array_equal(got, O.partial_target(lab, mask))
    masks = rng.integers(0, 2, (2, 15)).astype(np.int64)
    got = ops.partial_target(torch.from_numpy(lab).to(gpu), torch.from_numpy(masks)).cpu().numpy()
    ref = np.stack([O.partial_target(lab[i:i + 1], masks[i])[0] for i in range(2)])
    np.testing.assert_array_equal(got.reshape(ref.shape), ref)



def test_partial_target_every_supervise_mask_row(gpu):
    """A12 on the reference's own table (G14: the driver's lines run on all 240 rows of supervise_mask.csv, batch of
    two masked with one row as the driver does): the device pass is bit-exact for every row."""
    from loss_functions import losses
    g = golden("g14_partial_target.npz")
    lab = torch.from_numpy(g["labels"]).to(gpu)
    for i in range(len(g["names"])):
        got = losses.make_partial_target(lab, torch.from_numpy(g["masks"][i].astype(np.int64))).cpu().numpy()
        np.testing.assert_array_equal(got.astype(np.uint8), g["cmask"][i])
        assert got.dtype == np.float32 and got.shape == g["labels"].shape

# ------------------------------------------------------------- f2/f3: consistency branch of get_loss (G9)
@pytest.mark.parametrize("tag", ["mix", "none", "all"])
def test_g9_get_loss_consistency(gpu, tag):
    from loss_functions.losses import get_loss
    g = golden("g9_consistency.npz")
    lg = torch.from_numpy(g[f"{tag}_logits"]).to(gpu).requires_grad_(True)
    att = [torch.from_numpy(g[f"{tag}_att{i}"]).to(gpu).requires_grad_(True) for i in range(3)]
    attl = list(att)
    v, conf = get_loss(lg, 0, [], torch.from_numpy(g[f"{tag}_labels"]).to(gpu),
                       [torch.from_numpy(g[f"{tag}_mask"]).to(gpu)], None, attl,
                       torch.from_numpy(g[f"{tag}_refine"]).to(gpu), torch.from_numpy(g[f"{tag}_label_t"]),
                       weight_feature=0.07)
    assert len(attl) == 3 and conf == 0.10
    np.testing.assert_allclose(float(v), float(g[f"{tag}_value"]), rtol=1e-4)
    v.backward()
    ref = g[f"{tag}_dlogits"]
    np.testing.assert_allclose(lg.grad.cpu().numpy(), ref, rtol=1e-3, atol=1e-4 * np.abs(ref).max())
    for i in range(3):
        ref = g[f"{tag}_datt{i}"]
        got = att[i].grad.cpu().numpy() if att[i].grad is not None else np.zeros_like(ref)
        np.testing.assert_allclose(got, ref, rtol=1e-3, atol=1e-4 * max(np.abs(ref).max(), 1e-12))


def test_g9_edice_full2(gpu):
    from loss_functions.loss_partial import EDiceLoss_full2
    g = golden("g9_consistency.npz")
    t, m = torch.from_numpy(g["f2_t"]).to(gpu), torch.from_numpy(g["f2_m"]).to(gpu)
    for tag, kw in (("sig_m", dict(uce=False, mask=m)), ("sig_nom", dict(uce=False)),
                    ("id_m", dict(uce=False, mask=m, sigmoid=False)), ("sig_uce", dict(uce=True, mask=m))):
        xi = torch.from_numpy(g[f"f2_{tag}_in"]).to(gpu).requires_grad_(True)
        v = EDiceLoss_full2(2)(xi, t, **kw)
        np.testing.assert_allclose(float(v), float(g[f"f2_{tag}_value"]), rtol=1e-4)
        v.backward()
        ref = g[f"f2_{tag}_grad"]
        np.testing.assert_allclose(xi.grad.cpu().numpy(), ref, rtol=1e-3, atol=1e-4 * np.abs(ref).max())


def test_consistency_on_native_feam3_outputs(gpu):
    """End to end: feam3 (deep_up) outputs + a native refiner's output -> get_loss consistency branch, gradients
    through the attention maps into the model, against the oracle on the same values."""
    import unet3D
    from loss_functions.losses import get_loss
    torch.manual_seed(3)
    m = unet3D.unet3D_with_feam3([1, 2, 2, 2, 2], num_classes=14, weight_std=True, deep_up=True)
    apply_recipe(m, seed=0)
    m = m.to(gpu).train()
    x = torch.from_numpy(input_volume((1, 1, 32, 32, 32), seed=5, kind="normal")).to(gpu)
    logits, att, _, _ = m(x)
    refine = torch.randn(13, 2, 32, 32, 32, device=gpu) * 3
    lab = torch.from_numpy(label_volume((1, 1, 32, 32, 32), 14, seed=6)).to(gpu)
    mvec = torch.ones(15, dtype=torch.int64, device=gpu)
    lt = torch.tensor([1, 0, 0, 1, 0, 1, 1, 0, 0, 0, 1, 0, 0]).float()
    v, _ = get_loss(logits, 0, [], lab, [mvec], None, att, refine, lt, weight_feature=0.1)
    lgc = logits.detach().cpu().requires_grad_(True)
    atc = [a.detach().cpu().requires_grad_(True) for a in att]
    vr = O.get_loss_consistency(lgc, lab.cpu(), [mvec.cpu()], atc, refine.cpu(), lt, weight_feature=0.1)
    np.testing.assert_allclose(float(v), float(vr), rtol=1e-4)
    v.backward()
    vr.backward()
    assert torch.isfinite(m.eam21.kv.weight.grad).all() and m.eam21.kv.weight.grad.abs().sum() > 0


def test_inference_pack_cache_tracks_weight_updates(gpu):
    """no_grad forwards reuse the standardised weight packs only while the weights are unchanged: a native SGD
    step, an in-place torch update and load_state_dict each invalidate them (results equal an uncached run)."""
    import unet3D
    from u3d import ops
    from u3d.optim import SGD
    m = _model("baseline", C=16).to(gpu)
    x = torch.from_numpy(input_volume((1, 1, 16, 16, 16), seed=3, kind="ct")).to(gpu)

    def fwd():
        with torch.no_grad():
            return m.eval()(x).clone()

    def uncached():
        ops.PACK_CACHE_OK[0] = False
        try:
            return fwd()
        finally:
            ops.PACK_CACHE_OK[0] = True

    y0 = fwd()
    assert torch.equal(fwd(), y0)                                   # cache hit: same result
    m.train()
    opt = SGD(m.parameters(), lr=0.5, momentum=0.9)
    lg, _, _ = m(x)
    (lg.float() ** 2).mean().backward()
    opt.step()                                                      # native in-place update
    y1 = fwd()
    assert not torch.equal(y1, y0) and torch.equal(y1, uncached())
    with torch.no_grad():
        m.layer2[0].conv1.weight.mul_(1.5)                          # torch in-place update (version bump)
    y2 = fwd()
    assert not torch.equal(y2, y1) and torch.equal(y2, uncached())
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd["conv1.weight"].neg_()
    m.load_state_dict(sd)
    y3 = fwd()
    assert torch.equal(y3, uncached())


def test_g11_get_dice2(gpu):
    """The refiner's metric (train_amos_atlas_final.py:294) against the reference's own values (incl. exact ties)."""
    from evaluate_amos import get_dice2
    g = golden("g11_dice2.npz")
    d, se, sp, am = get_dice2(torch.from_numpy(g["refine"]).to(gpu), torch.from_numpy(g["labels"]).to(gpu), 1,
                              num_class=13)
    np.testing.assert_allclose([float(v) for v in d], g["dice"], atol=1e-6)
    np.testing.assert_allclose([float(v) for v in se], g["senc"], atol=1e-6)
    np.testing.assert_allclose([float(v) for v in sp], g["spec"], atol=1e-6)
    assert np.array_equal(am.cpu().numpy(), g["argmax"])
