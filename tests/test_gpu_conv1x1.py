"""bf16 1^3 convolution kernel (csrc/conv1x1.hip, u3d_conv1x1): forward stride 1 / 2 with the GroupNorm+ReLU
prologue, and the stride-1 data gradient, against an fp64 CPU reference on the same bf16-rounded operands (and the
bf16-rounded prologue), and against the implicit GEMM it replaces (U3D_CONV1X1=0 routing). Shapes: every 1^3 conv of
the trunk at reduced volume, channel counts with cx % 16 == 8 (half-filled last k step), co tiles split over the
grid (cy > 128), partial 32-voxel tiles, odd volumes at stride 2, several samples. Tolerance: bf16 output rounding,
1e-2 of max |y| (as test_gpu_bf16.py). Reference: F.conv3d(kernel 1, stride s) in Conv3d.forward (unet3D.py:27) via
the NoBottleneck downsample branch (:56-73, _make_layer :1666-1686)."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_bf16 import _act_ref, _bf

pytestmark = pytest.mark.gpu

CASES = [(2, 32, 64, (12, 10, 16), 2), (2, 64, 128, (8, 6, 10), 2), (2, 128, 256, (6, 6, 6), 2),
         (2, 256, 256, (4, 4, 4), 2), (2, 64, 32, (8, 8, 8), 1), (2, 128, 64, (6, 6, 6), 1),
         (2, 256, 128, (3, 3, 3), 1), (2, 256, 256, (3, 3, 3), 1), (3, 24, 40, (5, 7, 9), 2),
         (1, 40, 8, (9, 5, 3), 1), (1, 8, 200, (7, 3, 11), 2), (4, 32, 96, (1, 1, 37), 1)]


def _route(ops, on):
    saved = ops.USE_CONV1X1
    ops.USE_CONV1X1 = on
    return saved


@pytest.mark.parametrize("n,cx,cy,dims,s", CASES)
@pytest.mark.parametrize("gn", [True, False])
def test_conv1x1_fwd(gpu, n, cx, cy, dims, s, gn):
    from u3d import ops
    torch.manual_seed(cx + cy + s)
    x = (torch.randn((n,) + dims + (cx,), device=gpu) * 1.5 + 0.3).to(torch.bfloat16)
    w = torch.randn(cy, cx, 1, 1, 1, device=gpu)
    G = 8 if cx % 16 else 16
    st = ops.gn_stats(x, G) if gn else None
    ga = 1 + 0.1 * torch.randn(cx, device=gpu)
    be = 0.1 * torch.randn(cx, device=gpu)
    pf, pd, _ = ops.wstd_fwd(w, torch.bfloat16, True)
    g = (st, ga, be, G) if gn else None
    y = ops.conv_fwd(x, pf, cy, 1, s, g)
    a = _act_ref(x, st, ga, be, G).permute(0, 4, 1, 2, 3)
    wq = pf.float().cpu()[0, :cy, :cx].reshape(cy, cx, 1, 1, 1).double()
    ref = F.conv3d(a, wq, stride=s).permute(0, 2, 3, 4, 1)
    assert y.shape == ref.shape
    err = (y.double().cpu() - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err
    saved = _route(ops, False)
    try:
        y0 = ops.conv_fwd(x, pf, cy, 1, s, g)
    finally:
        _route(ops, saved)
    assert (y.double() - y0.double()).abs().max().item() < 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("n,cx,cy,dims,s", [c for c in CASES if c[4] == 1] + [(2, 64, 32, (16, 16, 16), 1)])
def test_conv1x1_dgrad_stride1(gpu, n, cx, cy, dims, s):
    """conv_dgrad of a stride-1 1^3 conv (cin = cx, cout = cy): dx = dy . W through the [cin_p][cout_p] pack."""
    from u3d import ops
    torch.manual_seed(7 + cx)
    w = torch.randn(cy, cx, 1, 1, 1, device=gpu)
    pf, pd, _ = ops.wstd_fwd(w, torch.bfloat16, True)
    dy = torch.randn((n,) + dims + (cy,), device=gpu).to(torch.bfloat16)
    dx = ops.conv_dgrad(dy, pd, cx, (n,) + dims, 1, 1)
    wq = pf.float().cpu()[0, :cy, :cx].reshape(cy, cx, 1, 1, 1).double()
    ref = torch.nn.grad.conv3d_input((n, cx) + dims, wq, _bf(dy.cpu().float()).permute(0, 4, 1, 2, 3)).permute(
        0, 2, 3, 4, 1)
    err = (dx.double().cpu() - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err


def test_conv1x1_bench_shapes(gpu):
    """The trunk's 1^3 convs at the bench size (2 x 96^3 input): 96^3 32 -> 48^3 64 (stride 2) and 48^3 64 -> 32
    (stride 1), sampled output planes against fp64."""
    from u3d import ops
    torch.manual_seed(3)
    for (cx, cy, s, dd) in [(32, 64, 2, 96), (64, 32, 1, 48)]:
        x = (torch.randn((2, dd, dd, dd, cx), device=gpu) * 1.2 - 0.4).to(torch.bfloat16)
        w = torch.randn(cy, cx, 1, 1, 1, device=gpu)
        st = ops.gn_stats(x, 16)
        ga = 1 + 0.1 * torch.randn(cx, device=gpu)
        be = 0.1 * torch.randn(cx, device=gpu)
        pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
        y = ops.conv_fwd(x, pf, cy, 1, s, (st, ga, be, 16))
        od = y.shape[1]
        wq = pf.float().cpu()[0, :cy, :cx].double()
        for n in range(2):
            for pd_ in (0, od // 2, od - 1):
                a = _act_ref(x[n:n + 1, s * pd_:s * pd_ + 1], st[n:n + 1], ga, be, 16)[0, 0]  # [h, w, cx]
                ref = torch.einsum("hwc,oc->hwo", a[::s, ::s], wq)
                err = (y[n, pd_].double().cpu() - ref).abs().max().item()
                assert err < 1e-2 * ref.abs().max().item(), (cx, cy, n, pd_, err)


@pytest.mark.parametrize("n,c,dims", [(2, 32, (12, 10, 16)), (2, 64, (8, 8, 8)), (3, 128, (5, 7, 9)), (1, 256, (4, 6, 3))])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_gn_bwd2_compact_stride2_da2(gpu, n, c, dims, dt):
    """gn_bwd2 with the downsample branch's data gradient kept at the stride-2 conv's output resolution equals
    gn_bwd2 on the zero-filled full-resolution tensor, bitwise (same arithmetic on the same values), including dx
    accumulation and the GN parameter gradients."""
    from u3d import ops
    torch.manual_seed(c)
    x = (torch.randn((n,) + dims + (c,), device=gpu) * 1.3 + 0.2).to(dt)
    da1 = torch.randn_like(x)
    od = tuple(ops.out_dim(d, 1, 2) for d in dims)
    da2c = torch.randn((n,) + od + (c,), device=gpu).to(dt)
    st = ops.gn_stats(x, 16)
    g1 = (1 + 0.1 * torch.randn(c, device=gpu), 0.1 * torch.randn(c, device=gpu))
    g2 = (1 + 0.1 * torch.randn(c, device=gpu), 0.1 * torch.randn(c, device=gpu))
    base = torch.randn_like(x)
    outs = []
    for compact in (True, False):
        dx = base.clone()
        dps = [(torch.zeros(c, device=gpu), torch.zeros(c, device=gpu)) for _ in range(2)]
        da2 = da2c if compact else ops.expand_s2(da2c, x.shape[:4])
        ops.gn_bwd2(da1, da2, x, st, g1, g2, 16, dx=dx, accumulate=True, dparams1=dps[0], dparams2=dps[1],
                    da2_s2=compact)
        outs.append((dx, dps))
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
