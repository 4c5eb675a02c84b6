"""The forward ring's normalised side output (round 6, u3d_conv32_ring_stats_xn): the 32->32 3^3 forward with the
GroupNorm + ReLU prologue also stores relu(gn(x)) — the values it stages — so the conv's weight gradient reads that
operand without re-normalising every staged piece (wgrad_ring_dma_kernel<false>). Checks, on ragged shapes (partial
8 x 32 plane tiles, so the tile / halo / volume masks all take both values) and at the bench size:
* y and the output GroupNorm(16) statistics bitwise those of u3d_conv32_ring_stats (the side store changes nothing);
* every voxel of xn equals relu(x * sc + sh) rounded to bf16 (fp32 fma, as the prologue computes it; a separate
  mul + add in the torch reference may round differently: <= 1 bf16 ulp, on at most 1e-4 of the entries);
* the weight gradient on xn without the GroupNorm prologue is BITWISE the weight gradient on x with it.
Reference: Conv3d.forward (unet3D.py:16-27) behind NoBottleneck's GroupNorm + ReLU (:44-53, :56-73)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(gpu, n, dims, seed, res):
    from u3d import ops
    torch.manual_seed(seed)
    x = (torch.randn((n,) + dims + (32,), device=gpu) * 1.3 + 0.2).to(torch.bfloat16)
    w = torch.randn(32, 32, 3, 3, 3, device=gpu)
    st = ops.gn_stats(x, 16)
    ga = 1 + 0.2 * torch.randn(32, device=gpu)
    be = 0.2 * torch.randn(32, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    r = torch.randn((n,) + dims + (32,), device=gpu).to(torch.bfloat16) if res else None
    dy = torch.randn((n,) + dims + (32,), device=gpu).to(torch.bfloat16)
    return x, pf, (st, ga, be, 16), r, dy


def _xn_ref(x, gn):
    st, ga, be, G = gn
    n, c = x.shape[0], x.shape[-1]
    g = torch.arange(c, device=x.device) // (c // G)
    sc = st[:, g, 1] * ga[None]
    sh = be[None] - st[:, g, 0] * sc
    a = x.float() * sc.view(n, 1, 1, 1, c) + sh.view(n, 1, 1, 1, c)
    return torch.clamp_min(a, 0).to(torch.bfloat16)


@pytest.mark.parametrize("n,dims,res", [(2, (20, 21, 45), False), (1, (11, 16, 70), True), (3, (9, 9, 33), True),
                                        (2, (96, 96, 96), True), (2, (96, 96, 96), False)])
def test_ring_xn_side_output(gpu, n, dims, res):
    from u3d import ops
    x, pf, gn, r, dy = _case(gpu, n, dims, 31 + n, res)
    ops.RING_XN = True  # (off by default: measured slower in the step)
    try:
        assert ops.ring_xn_ok(x, 32, 3, 1, gn)
    finally:
        ops.RING_XN = False
    y0, st0 = ops.conv_fwd_stats(x, pf, 32, 3, 1, gn, r)
    poison = torch.full_like(x, float("nan"))  # freed right away: xn's allocation reuses this block
    del poison
    y, st, xn = ops.conv_fwd_stats_xn(x, pf, 32, 3, 1, gn, r)
    assert torch.equal(y, y0), "the side store changed the conv output"
    assert torch.equal(st, st0), "the side store changed the output statistics"
    ref = _xn_ref(x, gn)
    diff = (xn.float() - ref.float()).abs()
    ulp = torch.maximum(ref.float().abs(), xn.float().abs()) * 2.0 ** -7 + 1e-6
    assert bool(torch.isfinite(xn.float()).all()), "unwritten (garbage) voxels in xn"
    assert bool((diff <= ulp).all()), f"xn off by more than one bf16 ulp: max {diff.max().item():.3e}"
    assert (diff > 0).float().mean().item() <= 1e-4
    p0, ns0 = ops.conv_wgrad(dy, x, 3, 1, gn)
    p0 = p0[:ns0].clone()  # (the slabs live in a reused workspace)
    p1, ns1 = ops.conv_wgrad(dy, xn, 3, 1, None)
    assert ns0 == ns1 and torch.equal(p0, p1[:ns1]), "weight gradient on xn differs from the GN form"
