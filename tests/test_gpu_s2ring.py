"""The stride-2 3^3 forward as an input-plane walk (round 5, u3d_conv_s2_ring: layer1.0.conv1 of the 96^3 trunk, 32 -> 64
channels with the GroupNorm + ReLU prologue) against an fp64 reference on the same bf16-rounded operands (the GN + ReLU
prologue rounded to bf16 as the kernel stages it): max error per output plane <= 1e-2 of the tensor's max |y| and
rel L2 <= 4e-3 (bf16 output rounding), the output GroupNorm(16) statistics against the statistics pass on the stored
output, and at the bench size against the implicit GEMM it replaces. Reference: NoBottleneck.conv1 with stride 2,
unet3D.py:45 (Conv3d :16-27), GroupNorm + ReLU :44-53."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _case(gpu, n, dims, seed, off=0.3):
    from u3d import ops
    torch.manual_seed(seed)
    x = (torch.randn((n,) + dims + (32,), device=gpu) * 1.5 + off).to(torch.bfloat16)
    w = torch.randn(64, 32, 3, 3, 3, device=gpu)
    st = ops.gn_stats(x, 16)
    ga = 1 + 0.1 * torch.randn(32, device=gpu)
    be = 0.1 * torch.randn(32, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    return x, pf, (st, ga, be, 16)


def _ref(x, pf, gn):
    st, ga, be, G = gn
    xf = x.float().cpu()
    n, c = xf.shape[0], xf.shape[-1]
    g = torch.arange(c) // (c // G)
    s = st.cpu()
    sc = s[:, g, 1] * ga.cpu()[None]
    sh = be.cpu()[None] - s[:, g, 0] * sc
    a = torch.clamp_min(torch.addcmul(sh.view(n, 1, 1, 1, c), xf, sc.view(n, 1, 1, 1, c)), 0)
    a = a.to(torch.bfloat16).double().permute(0, 4, 1, 2, 3)
    wq = pf.float().cpu()[:, :64, :32].permute(1, 2, 0).reshape(64, 32, 3, 3, 3).double()
    return F.conv3d(a, wq, stride=2, padding=1).permute(0, 2, 3, 4, 1)


@pytest.mark.parametrize("n,dims,off", [(2, (24, 24, 24), 0.3), (1, (13, 18, 35), -0.5), (3, (16, 40, 20), 1.0),
                                        (2, (9, 33, 17), 0.0)])
def test_s2_ring_vs_fp64(gpu, n, dims, off):
    from u3d import ops
    x, pf, gn = _case(gpu, n, dims, 21, off)
    assert ops.query("u3d_conv_s2_ring_ok", n, 32, *dims, 64) == 1
    y, st = ops.conv_fwd_stats(x, pf, 64, 3, 2, gn)
    assert st is not None, "the stride-2 ring did not run"
    ref = _ref(x, pf, gn)
    got = y.double().cpu()
    assert got.shape == ref.shape
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 1e-2 * scale
    assert ((got - ref).norm() / ref.norm()).item() <= 4e-3
    st2 = ops.gn_stats(y, 16)
    ysc = y.float().abs().max().item()
    assert (st[..., 0] - st2[..., 0]).abs().max().item() < 1e-4 * ysc
    assert ((st[..., 1] - st2[..., 1]).abs() / st2[..., 1]).max().item() < 5e-4
    y2, st3 = ops.conv_fwd_stats(x, pf, 64, 3, 2, gn)  # deterministic, counter left at zero
    assert torch.equal(y, y2) and torch.equal(st, st3)


def test_s2_ring_bench_size_vs_implicit_gemm(gpu, monkeypatch):
    """2 x 96^3 x 32 -> 48^3 x 64 (the bench step's layer1.0.conv1): against the implicit GEMM it replaces (both bf16
    operands, fp32 accumulation in another order): rel L2 <= 4e-3, max <= 1e-2 of max |y|."""
    from u3d import ops
    x, pf, gn = _case(gpu, 2, (96, 96, 96), 22)
    y, st = ops.conv_fwd_stats(x, pf, 64, 3, 2, gn)
    assert st is not None
    monkeypatch.setattr(ops, "S2_RING", False)
    y0, st0 = ops.conv_fwd_stats(x, pf, 64, 3, 2, gn)
    assert st0 is None
    a, b = y.float(), y0.float()
    assert ((a - b).norm() / b.norm()).item() <= 4e-3
    assert (a - b).abs().max().item() <= 1e-2 * b.abs().max().item()
    st2 = ops.gn_stats(y, 16)
    assert ((st[..., 1] - st2[..., 1]).abs() / st2[..., 1]).max().item() < 5e-4
