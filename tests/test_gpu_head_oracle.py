"""The head's whole backward through the fused kernels against the oracle in fp64 (the fused
head + loss backward was checked only bitwise against the two-pass form).

precls_conv = GroupNorm(16, 32) -> ReLU -> Conv3d 1^3 + bias (unet3D.py:629-633 / :1653-1657, oracle.precls) followed
by EDiceLoss_partial (loss_partial.py:59-99, oracle.edice_partial); the oracle's autograd in fp64 on the same bf16 head
input gives the reference gradients of the head input, the GroupNorm affine parameters, the conv weight and its bias.
The native path: u3d_head_fwd -> u3d_partial_loss_fwd -> u3d_head_loss_bwd[_gn] (loss gradient, dA, bf16 dy, bias
partials and — v % 32 == 0 — the GroupNorm-backward partials in one pass) -> u3d_gn_bwd_parts (or u3d_gn_bwd) and the
1^3 weight gradient. Tolerances: the loss within 1e-3 and the bias gradient within 1e-2 (the logits come from the
bf16 forward); dA and the
weight-gradient operands are bf16, so dx / dgamma / dbeta / dW are held to 2e-2 of their largest magnitude
elementwise and 1e-2 in relative Frobenius norm. The backward alone is checked tighter against the oracle's loss
gradient on the kernel's own fp32 logits (loss and bias gradient 1e-5; dA within its bf16 GEMM operands'
rounding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _max_rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("S,dims,fused", [(2, (8, 8, 16), True), (1, (4, 8, 32), True), (3, (5, 6, 7), False),
                                          (2, (8, 8, 16), False)])
def test_head_backward_vs_oracle(gpu, S, dims, fused, monkeypatch):
    from oracle import ref_cpu as ref
    from u3d import ops
    monkeypatch.setattr(ops, "HEAD_GN_PARTS", fused)
    g = torch.Generator().manual_seed(17 + S)
    C, cin, G = 16, 32, 16
    x0 = (torch.randn((S,) + dims + (cin,), generator=g) * 1.3 + 0.2).to(torch.bfloat16)
    ga = 1 + 0.3 * torch.randn(cin, generator=g)
    be = 0.3 * torch.randn(cin, generator=g)
    W = 0.2 * torch.randn(C, cin, 1, 1, 1, generator=g)
    b = 0.1 * torch.randn(C, generator=g)
    lab = torch.randint(0, C, (S,) + dims, generator=g).float()
    wt = (torch.rand(C, generator=g) < 0.7).float()
    wt[0] = 1.0

    # ---- oracle, fp64 autograd on the same bf16 input values
    xr = x0.double().permute(0, 4, 1, 2, 3).contiguous().requires_grad_(True)
    gar, ber = ga.double().requires_grad_(True), be.double().requires_grad_(True)
    Wr, br = W.double().requires_grad_(True), b.double().requires_grad_(True)
    P = {"precls_conv.0.weight": gar, "precls_conv.0.bias": ber, "precls_conv.2.weight": Wr, "precls_conv.2.bias": br}
    loss_r = ref.edice_partial(ref.precls(P, xr, G), lab.double(), mask=[wt.double()])
    loss_r.backward()

    # ---- native
    xg, gag, beg, bg = x0.to(gpu), ga.to(gpu), be.to(gpu), b.to(gpu)
    labg, wtg = lab.to(gpu), wt.to(gpu)
    pf, pd, _ = ops.wstd_fwd(W.to(gpu), torch.bfloat16, False)
    st = ops.gn_stats(xg, G)
    gn = (st, gag, beg, G)
    lg = ops.head_fwd(xg, pf, C, bg, gn)
    loss, sums = ops.partial_loss_fwd(lg, labg, wtg, True, True)
    go = torch.ones(1, device=gpu)
    db = torch.empty(C, device=gpu)
    used_fused = ops.head_gn_parts_ok(lg, xg, cin, gn)
    assert used_fused == (fused and (lg.numel() // (C * S)) % 32 == 0)
    dg, dbt = torch.empty(cin, device=gpu), torch.empty(cin, device=gpu)
    if used_fused:
        dA, dyT, parts = ops.head_loss_bwd(lg, labg, wtg, sums, go, pd, cin, dbias=db, x0=xg, gn=gn)
        dx = ops.gn_bwd_parts(dA, xg, parts, st, gag, beg, G, dgamma=dg, dbeta=dbt)
    else:
        dA, dyT = ops.head_loss_bwd(lg, labg, wtg, sums, go, pd, cin, dbias=db)
        dx = ops.gn_bwd(dA, xg, st, gag, beg, G, dgamma=dg, dbeta=dbt)
    part, ns = ops.conv_wgrad(dyT, xg, 1, 1, gn)
    dW = part[:ns].sum(0)[0, :C, :cin]
    torch.cuda.synchronize()

    # (1) the backward alone: the oracle's loss gradient in fp64 on OUR fp32 logits. The bias gradient is a sum of fp32
    # loss-gradient values (1e-5); dA = dlogits W with the bf16 GEMM operands (dlogits and W rounded to bf16, fp32
    # accumulation, bf16 result): within 2^-7 of sum_c |dlogits_c W_c| per element
    lgr = lg.double().cpu().permute(0, 4, 1, 2, 3).contiguous().requires_grad_(True)
    loss_l = ref.edice_partial(lgr, lab.double(), mask=[wt.double()])
    assert abs(loss.item() - loss_l.item()) <= 1e-5 * abs(loss_l.item())
    (dl,) = torch.autograd.grad(loss_l, lgr)
    assert _max_rel(db.cpu(), dl.sum((0, 2, 3, 4))) <= 1e-5
    Wb = W.reshape(C, cin).to(torch.bfloat16).double()
    dlc = dl.permute(0, 2, 3, 4, 1)
    dA_ref = dlc @ Wb
    bound = 2.0 ** -7 * (dlc.abs() @ Wb.abs()) + 1e-9
    assert bool(((dA.cpu().double() - dA_ref).abs() <= bound).all())
    # (2) end to end against the oracle from the same bf16 input (the forward's bf16 operands included)
    assert abs(loss.item() - loss_r.item()) <= 1e-3 * abs(loss_r.item())
    assert _max_rel(db.cpu(), br.grad) <= 1e-2
    ref_dx = xr.grad.permute(0, 2, 3, 4, 1)
    for name, got, want in (("dx", dx.cpu(), ref_dx), ("dgamma", dg.cpu(), gar.grad), ("dbeta", dbt.cpu(), ber.grad),
                            ("dW", dW.cpu(), Wr.grad.reshape(C, cin))):
        assert _max_rel(got, want) <= 2e-2, (name, _max_rel(got, want))
        assert _rel(got, want) <= 1e-2, (name, _rel(got, want))
