"""GroupNorm statistics accumulated in the epilogue of the kernel that produces the activation (csrc/gnpart.h):
the decoder's upsample + skip (u3d_upsample2x_add_stats) and the stem conv (u3d_stem_fwd_stats). Each must store
exactly what the plain kernel stores (bitwise) and return the GroupNorm(16) statistics of that stored output as the
separate statistics pass computes them (u3d_gn_stats: shifted fp32 partials, fp64 combine): |d mean| <= 1e-5 x the
group's std, |d rstd| / rstd <= 1e-5 (fp64 epilogue sums vs the shifted pass). Shapes include the bench size
(2 x 96^3 output) and volumes whose blocks straddle samples. Reference: nn.GroupNorm(16, C) (unet3D.py:44-53) on
the outputs of nn.Upsample + skip (:1646, :1764-1783) and conv1 (:1632)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _check_stats(st, ref):
    mean_r, rstd_r = ref[..., 0].double(), ref[..., 1].double()
    dm = ((st[..., 0].double() - mean_r).abs() * rstd_r).max().item()
    dr = ((st[..., 1].double() - rstd_r).abs() / rstd_r).max().item()
    assert dm <= 1e-5 and dr <= 1e-5, (dm, dr)


@pytest.mark.parametrize("n,c,dims,skip", [(2, 32, (48, 48, 48), True), (2, 64, (24, 24, 24), True),
                                           (2, 128, (12, 12, 12), True), (2, 256, (6, 6, 6), True),
                                           (3, 16, (5, 7, 9), False), (1, 256, (3, 4, 5), True)])
def test_upsample_epilogue_stats(gpu, n, c, dims, skip, monkeypatch):
    from u3d import ops
    monkeypatch.setattr(ops, "UP_STATS_MAX_BYTES", 1 << 40)
    monkeypatch.setattr(ops, "EPI_STATS", True)
    torch.manual_seed(1)
    x = (torch.randn((n,) + dims + (c,), device=gpu) * 1.3 + 0.7).to(torch.bfloat16)
    od = tuple(2 * v for v in dims)
    sk = (torch.randn((n,) + od + (c,), device=gpu) - 2.0).to(torch.bfloat16) if skip else None
    y, st = ops.upsample2x_add_stats(x, sk)
    assert st is not None
    assert torch.equal(y, ops.upsample2x_add(x, sk))
    _check_stats(st, ops.gn_stats(y, 16))
    y2, st2 = ops.upsample2x_add_stats(x, sk)   # the counters / partials are left reusable
    assert torch.equal(st, st2)


@pytest.mark.parametrize("n,dims", [(2, (96, 96, 96)), (3, (5, 9, 64)), (1, (7, 6, 12)), (4, (4, 8, 32))])
def test_stem_epilogue_stats(gpu, n, dims, monkeypatch):
    from u3d import ops
    monkeypatch.setattr(ops, "STEM_STATS", True)
    torch.manual_seed(2)
    x = torch.rand((n, 1) + dims, device=gpu) * 2 - 1
    w = torch.randn(32, 1, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    d, h, w_ = dims
    if d * h * (w_ // 4) < 256:
        y, st = ops.stem_fwd_stats(x, pf, 32, 1, torch.bfloat16)
        assert st is None
        return
    y, st = ops.stem_fwd_stats(x, pf, 32, 1, torch.bfloat16)
    assert st is not None
    # the plain bf16 conv1 runs on the MFMA kernel (bf16-rounded input), the statistics variant on the fp32-input VALU
    # kernel: same output within bf16 rounding
    yp = ops.stem_fwd(x, pf, 32, 1, torch.bfloat16)
    assert (y.float() - yp.float()).abs().max().item() <= 1e-2 * yp.float().abs().max().item()
    _check_stats(st, ops.gn_stats(y, 16))
    _, st2 = ops.stem_fwd_stats(x, pf, 32, 1, torch.bfloat16)
    assert torch.equal(st, st2)
