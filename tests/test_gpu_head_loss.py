"""The partial loss's gradient formed inside the head's backward (u3d_head_loss_bwd, loss.DeferredLossGrad): the same
dA, bf16 dy and bias gradient as partial_loss_bwd + head_bwd bit for bit, the same parameter gradients for the whole
step, and every other reader of the logits' gradient (a second loss term, a hook, autograd.grad) sees the formed
tensor."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cin,dims", [(32, (2, 7, 9, 11)), (32, (2, 16, 16, 16)), (64, (1, 5, 6, 7)),
                                      (16, (3, 4, 4, 5)), (32, (1, 1, 1, 3))])
def test_head_loss_bwd_bitwise(gpu, cin, dims):
    from u3d import ops
    g = torch.Generator().manual_seed(3)
    lg = (torch.randn(dims + (16,), generator=g) * 3).to(gpu)
    lab = torch.randint(0, 16, dims, generator=g).float().to(gpu)
    wt = (torch.rand(16, generator=g) < 0.7).float().to(gpu)
    _, sums = ops.partial_loss_fwd(lg, lab, wt, True, True)
    go = torch.tensor([0.73], device=gpu)
    w = torch.randn(16, cin, 1, 1, 1, generator=g).to(gpu)
    _, pd, _ = ops.wstd_fwd(w, torch.bfloat16, False)
    db0, db1 = torch.empty(16, device=gpu), torch.empty(16, device=gpu)
    dl = ops.partial_loss_bwd(lg, lab, wt, sums, go, True, True)
    dA0, dy0 = ops.head_bwd(dl, pd, cin, dbias=db0)
    dA1, dy1 = ops.head_loss_bwd(lg, lab, wt, sums, go, pd, cin, dbias=db1)
    assert torch.equal(dA0, dA1)
    assert torch.equal(dy0, dy1)
    assert torch.equal(db0, db1)


def _step_grads(dev, fused, extra, monkeypatch, calls, gn_parts=False):
    import unet3D
    from loss_functions.loss_partial import EDiceLoss_partial
    from u3d import ops
    monkeypatch.setattr(ops, "HEAD_LOSS_FUSED", fused)
    monkeypatch.setattr(ops, "HEAD_GN_PARTS", gn_parts)
    torch.manual_seed(0)
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(dev).train()
    crit = EDiceLoss_partial(16)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand((2, 1, 32, 32, 32), generator=g) * 2 - 1).to(dev)
    lab = torch.randint(0, 16, (2, 32, 32, 32), generator=g).float().to(dev)
    mask = (torch.rand(16, generator=g) < 0.7).long().to(dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg, _, _ = m(x)
    loss = crit(lg, lab, mask=[mask])
    seen = []
    if extra == "sum":  # a second consumer of the logits: autograd sums the two gradients
        loss = loss + 0.05 * lg.square().mean()
    elif extra == "hook":
        lg.register_hook(lambda t: seen.append(t.double().abs().sum().item()))
    n0 = calls[0]
    loss.backward()
    torch.cuda.synchronize()
    return {n: p.grad.clone() for n, p in m.named_parameters()}, calls[0] - n0, seen


@pytest.mark.parametrize("extra", [None, "sum", "hook"])
def test_step_gradients_bitwise(gpu, monkeypatch, extra):
    from u3d import ops
    calls = [0]
    real = ops.head_loss_bwd

    def counted(*a, **k):
        calls[0] += 1
        return real(*a, **k)
    monkeypatch.setattr(ops, "head_loss_bwd", counted)
    a, na, sa = _step_grads(gpu, False, extra, monkeypatch, calls)
    b, nb, sb = _step_grads(gpu, True, extra, monkeypatch, calls)
    assert na == 0
    assert nb == (1 if extra is None else 0)  # any other reader forms the gradient first: the two-pass path runs
    assert sa == sb
    for n in a:
        assert torch.equal(a[n], b[n]), n


def test_autograd_grad_on_logits_is_formed(gpu):
    import unet3D
    from loss_functions.loss_partial import EDiceLoss_partial
    from u3d import ops
    from u3d.loss import ndhwc_view
    torch.manual_seed(1)
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(gpu).train()
    g = torch.Generator().manual_seed(9)
    x = (torch.rand((1, 1, 16, 16, 16), generator=g) * 2 - 1).to(gpu)
    lab = torch.randint(0, 16, (1, 16, 16, 16), generator=g).float().to(gpu)
    lg, _, _ = m(x)
    loss = EDiceLoss_partial(16)(lg, lab, mask=[torch.ones(16, dtype=torch.long, device=gpu)])
    (gl,) = torch.autograd.grad(loss, lg)
    lgv = ndhwc_view(lg.detach())
    _, sums = ops.partial_loss_fwd(lgv, lab, torch.ones(16, device=gpu), True, True)
    ref = ops.partial_loss_bwd(lgv, lab, torch.ones(16, device=gpu), sums, torch.ones(1, device=gpu), True, True)
    assert torch.equal(gl.permute(0, 2, 3, 4, 1), ref)


@pytest.mark.parametrize("dims", [(2, 7, 9, 11), (1, 16, 16, 16), (2, 1, 1, 5), (2, 40, 40, 40)])
def test_loss_forward_lane_pair_form(gpu, dims):
    """The 16-class softmax + BCE forward with each voxel's classes over a lane pair (LOSS_PAIR) against the one-lane
    form: the same loss and per-class sums up to the fp32 partial-sum order; deterministic."""
    from u3d import ops
    g = torch.Generator().manual_seed(11)
    lg = (torch.randn(dims + (16,), generator=g) * 4).to(gpu)
    lab = torch.randint(0, 16, dims, generator=g).float().to(gpu)
    wt = (torch.rand(16, generator=g) < 0.7).float().to(gpu)
    l1, s1 = ops.partial_loss_fwd(lg, lab, wt, True, True)
    l1b, s1b = ops.partial_loss_fwd(lg, lab, wt, True, True)
    assert torch.equal(l1, l1b) and torch.equal(s1, s1b)
    with ops.option("LOSS_PAIR", 0):
        l0, s0 = ops.partial_loss_fwd(lg, lab, wt, True, True)
    # fp32 per-block partials of up to a few thousand terms, summed in a different order: ~1e-6 relative apart
    torch.testing.assert_close(s1, s0, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(l1, l0, rtol=2e-5, atol=1e-7)


def _gn_case(gpu, dims, cin=32, G=8, seed=4):
    from u3d import ops
    g = torch.Generator().manual_seed(seed)
    lg = (torch.randn(dims + (16,), generator=g) * 3).to(gpu)
    lab = torch.randint(0, 16, dims, generator=g).float().to(gpu)
    wt = (torch.rand(16, generator=g) < 0.7).float().to(gpu)
    _, sums = ops.partial_loss_fwd(lg, lab, wt, True, True)
    go = torch.tensor([0.61], device=gpu)
    w = torch.randn(16, cin, 1, 1, 1, generator=g).to(gpu)
    _, pd, _ = ops.wstd_fwd(w, torch.bfloat16, False)
    x0 = (torch.randn(dims + (cin,), generator=g) * 1.4 + 0.3).to(gpu).to(torch.bfloat16)
    st = ops.gn_stats(x0, G)
    ga = (1 + 0.3 * torch.randn(cin, generator=g)).to(gpu)
    be = (0.3 * torch.randn(cin, generator=g)).to(gpu)
    return lg, lab, wt, sums, go, pd, x0, (st, ga, be, G)


@pytest.mark.parametrize("dims,G", [((2, 8, 8, 16), 8), ((3, 5, 6, 32), 16), ((1, 1, 4, 8), 8), ((2, 96, 96, 96), 8),
                                    ((1, 32, 33, 35), 4)])
def test_head_loss_bwd_gn_parts(gpu, dims, G):
    """u3d_head_loss_bwd_gn (round 6): the head's GN + ReLU prologue backward partials taken in the head's pass.
    dA and the bf16 dy bitwise those of u3d_head_loss_bwd; the bias gradient, the partials (against an fp64 torch
    restatement of gn_bwd's per-channel sums, reference: GroupNorm backward behind unet3D.py:1644-1657) and the
    resulting dx / dgamma / dbeta (against the separate-partial-pass gn_bwd) within fp32 summation-order tolerance."""
    from u3d import ops
    lg, lab, wt, sums, go, pd, x0, gn = _gn_case(gpu, dims, G=G)
    assert ops.head_gn_parts_ok(lg, x0, 32, gn)
    db0, db1 = torch.empty(16, device=gpu), torch.empty(16, device=gpu)
    dA0, dy0 = ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, dbias=db0)
    dA1, dy1, parts = ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, dbias=db1, x0=x0, gn=gn)
    assert torch.equal(dA0, dA1) and torch.equal(dy0, dy1)
    torch.testing.assert_close(db1, db0, rtol=1e-5, atol=1e-6)
    # fp64 restatement of the per-(sample, channel) sums
    st, ga, be, _ = gn
    n, c = x0.shape[0], 32
    grp = torch.arange(c, device=gpu) // (c // G)
    mu, rs = st[:, grp, 0].double(), st[:, grp, 1].double()
    xf = x0.double().reshape(n, -1, c)
    sc = rs.float() * ga[None]
    pre = x0.float().reshape(n, -1, c) * sc[:, None] + (be[None] - st[:, grp, 0] * sc)[:, None]
    gmask = torch.where(pre > 0, dA0.double().reshape(n, -1, c), torch.zeros((), dtype=torch.float64, device=gpu))
    xhat = (xf - mu[:, None]) * rs[:, None]
    ref = torch.stack([gmask.sum(1), (gmask * xhat).sum(1)], -1)  # [n, c, 2]
    got = parts.double().sum(1)
    scale = gmask.abs().sum(1).max().item() + 1e-30
    assert (got - ref).abs().max().item() <= 1e-5 * scale, (got - ref).abs().max().item()
    dg0, dbt0 = torch.empty(c, device=gpu), torch.empty(c, device=gpu)
    dg1, dbt1 = torch.empty(c, device=gpu), torch.empty(c, device=gpu)
    dx0 = ops.gn_bwd(dA0, x0, st, ga, be, G, dgamma=dg0, dbeta=dbt0)
    dx1 = ops.gn_bwd_parts(dA1, x0, parts, st, ga, be, G, dgamma=dg1, dbeta=dbt1)
    torch.testing.assert_close(dg1, dg0, rtol=1e-4, atol=1e-4 * dg0.abs().max().item())
    torch.testing.assert_close(dbt1, dbt0, rtol=1e-4, atol=1e-4 * dbt0.abs().max().item())
    # bf16 dx: the apply coefficients differ in the last fp32 bits -> at most one bf16 rounding step apart
    d = (dx1.float() - dx0.float()).abs()
    ulp = torch.maximum(dx0.float().abs(), dx1.float().abs()) * 2.0 ** -7 + 1e-6
    assert bool((d <= ulp).all()), d.max().item()
    # deterministic; the bias gradient's arrival counter is left zeroed (a second launch sums the same rows)
    db2 = torch.full((16,), float("nan"), device=gpu)
    _, _, parts2 = ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, dbias=db2, x0=x0, gn=gn)
    assert torch.equal(parts, parts2) and torch.equal(db1, db2)


def test_head_loss_bwd_gn_dbias_last_arriver(gpu, monkeypatch):
    """The GN head backward's bias gradient summed in-kernel by the last-arriving workgroup (round 6) against the two
    channel-sum launches it replaces: fp64 sums of the same partial rows, so equal to fp32 rounding."""
    from u3d import ops
    lg, lab, wt, sums, go, pd, x0, gn = _gn_case(gpu, (2, 64, 64, 64), G=8)
    db0, db1 = torch.empty(16, device=gpu), torch.empty(16, device=gpu)
    monkeypatch.setattr(ops, "HEAD_DBIAS_FUSED", False)
    ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, dbias=db0, x0=x0, gn=gn)
    monkeypatch.setattr(ops, "HEAD_DBIAS_FUSED", True)
    for _ in range(3):
        ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, dbias=db1, x0=x0, gn=gn)
        torch.testing.assert_close(db1, db0, rtol=1e-6, atol=1e-6 * db0.abs().max().item())


def test_head_loss_bwd_gn_applicability(gpu):
    from u3d import ops
    lg, lab, wt, sums, go, pd, x0, gn = _gn_case(gpu, (2, 3, 5, 7))  # v = 105: blocks would straddle samples
    assert not ops.head_gn_parts_ok(lg, x0, 32, gn)
    with pytest.raises(AssertionError):
        ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, x0=x0, gn=gn)


def test_step_gradients_head_gn_parts(gpu, monkeypatch):
    """Whole-step parameter gradients with the head's GN partials fused vs the separate partial pass: the same up to
    fp32 summation order (the partial sums are regrouped; everything upstream inherits the last-bit differences)."""
    calls = [0]
    a, _, _ = _step_grads(gpu, True, None, monkeypatch, calls, gn_parts=False)
    b, _, _ = _step_grads(gpu, True, None, monkeypatch, calls, gn_parts=True)
    for n in a:
        scale = a[n].abs().max().item() + 1e-12
        err = (a[n] - b[n]).abs().max().item()
        assert err <= 2e-2 * scale, (n, err, scale)
