"""GroupNorm backward fused into the small-volume data gradient (round 5: u3d_conv_small_dgrad_gn, then
u3d_gn_bwd_apply_coef) against the separate form (conv_dgrad + gn_bwd): dA bitwise equal (same kernel, same slab
order), dgamma / dbeta / dx equal up to fp32 reassociation of the per-channel sums (the partial pass reduces the same
terms per block, here per brick), deterministic run to run. The 12^3 / 6^3 levels of the trunk (layer3, layer4, the
x8 decoder block). Reference: autograd of NoBottleneck's relu(gn(x)) -> conv3x3x3 (unet3D.py:44-73)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # n, d, h, w, cin (x, dA), cout (dy), groups, x offset
    (2, 12, 12, 12, 256, 256, 16, 0.0),   # layer3 / x8_resb
    (2, 6, 6, 6, 256, 256, 16, 0.0),      # layer4
    (2, 12, 12, 12, 128, 256, 16, 0.0),   # cin != cout
    (1, 12, 12, 12, 256, 256, 16, 30.0),  # n = 1, |mean| / std ~ 40
    (3, 8, 8, 8, 64, 64, 8, 0.0),         # n = 3, 8 channels per group
]


def _setup(gpu, n, d, h, w, cin, cout, groups, off):
    from u3d import ops
    torch.manual_seed(7)
    x = (torch.randn((n, d, h, w, cin), device=gpu) * 0.8 + 0.2 + off).to(torch.bfloat16)
    dy = (torch.randn((n, d, h, w, cout), device=gpu) * 0.3).to(torch.bfloat16)
    wt = torch.randn((cout, cin, 3, 3, 3), device=gpu) * 0.05
    (pf, pd, st), = ops.wstd_fwd_batch([(wt, True, True)], torch.bfloat16)
    gn = (ops.gn_stats(x, groups), 1 + 0.1 * torch.randn(cin, device=gpu), 0.1 * torch.randn(cin, device=gpu), groups)
    return x, dy, pd, gn


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:4])) + f"_c{c[4]}-{c[5]}_g{c[6]}_o{c[7]:g}")
def test_small_dgrad_gn_matches_separate(gpu, case):
    from u3d import ops
    x, dy, pd, gn = _setup(gpu, *case)
    cin = x.shape[-1]
    da = ops.conv_dgrad(dy, pd, cin, tuple(x.shape[:4]), 3, 1)
    dg0, db0 = torch.zeros(cin, device=gpu), torch.zeros(cin, device=gpu)
    dx0 = ops.gn_bwd(da, x, gn[0], gn[1], gn[2], gn[3], dgamma=dg0, dbeta=db0)
    outs = []
    for _ in range(2):
        dg, db = torch.full((cin,), 7.0, device=gpu), torch.full((cin,), 7.0, device=gpu)  # overwritten, not added to
        r = ops.conv_dgrad_gn(dy, pd, cin, x, 3, 1, gn, dgb=lambda: (dg, db))
        assert r is not None and isinstance(r[1], tuple) and r[1][0] == "coef", "the fused small path did not run"
        dx = ops.gn_bwd_apply_coef(r[0], x, r[1][1], gn[3])
        outs.append((r[0], dx, dg, db, r[1][1]))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], da)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)  # deterministic (and the arrival counters were left at zero)
    _, dx, dg, db, coef = outs[0]
    for a, b in ((dg0, dg), (db0, db)):
        err = ((a - b).norm() / a.norm().clamp_min(1e-12)).item()
        assert err < 2e-5, err
    err = ((dx0.float() - dx.float()).norm() / dx0.float().norm()).item()
    assert err < 2e-3, err
    # accumulate into an existing gradient
    base = (torch.randn_like(x.float()) * 0.1).to(torch.bfloat16)
    acc = ops.gn_bwd_apply_coef(outs[0][0], x, coef, gn[3], dx=base.clone(), accumulate=True)
    ref = base.float() + dx0.float()
    assert ((acc.float() - ref).norm() / ref.norm()).item() < 4e-3
