"""GroupNorm backward with its partial pass fused into the persistent brick data gradient's epilogue
(ops.conv_dgrad_gn -> u3d_convg_brick_dgrad_gn, then ops.gn_bwd_parts) against the separate form (conv_dgrad +
gn_bwd): dA bitwise equal (same kernel schedule, same stores), dx / dgamma / dbeta equal up to fp32 reassociation of
the per-channel sums, deterministic run to run. The 48^3 / 24^3 levels of the trunk.
Reference: autograd of NoBottleneck's relu(gn(x)) -> conv3x3x3 (unet3D.py:44-73)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _every_size(monkeypatch):
    """the trunk routes only small volumes through the fused form (ops.GN_BWD_FUSED_BRICK_MAX_VOX); the kernel is
    tested at every size"""
    from u3d import ops
    monkeypatch.setattr(ops, "GN_BWD_FUSED_BRICK_MAX_VOX", 1 << 40)

CASES = [  # n, d, h, w, cin (x, dA), cout (dy), groups, x offset
    (2, 48, 48, 48, 64, 64, 16, 0.0),     # 48^3 level: 16-wide bricks, 64-channel tiles
    (2, 24, 24, 24, 128, 128, 16, 0.0),   # 24^3 level: 8-wide bricks, two 64-channel tiles
    (2, 16, 32, 32, 64, 64, 16, 0.0),     # 32-channel co tiles (64-channel ones give < 128 workgroups)
    (2, 21, 26, 37, 64, 64, 16, 0.0),     # ragged bricks (partial in every dimension)
    (2, 24, 24, 24, 64, 128, 8, 0.0),     # cin != cout, 8 channels per group
    (2, 24, 24, 24, 64, 64, 16, 40.0),    # |mean| / std ~ 50: the (x - mean) form of the sums
    # the epilogue's two-slot GroupNorm table (indexed by sample parity) and the padded-channel masks
    (1, 32, 32, 32, 64, 64, 16, 0.0),     # n = 1
    (3, 16, 24, 24, 64, 64, 16, 0.0),     # n = 3: workgroups whose brick runs cross sample boundaries
    (2, 24, 24, 24, 48, 64, 8, 0.0),      # dA channels 48: a partially padded 32-channel tile, 6 per group
    (2, 16, 32, 32, 40, 64, 8, 3.0),      # dA channels 40, 5 per group
]


def _setup(gpu, n, d, h, w, cin, cout, groups, off):
    from u3d import ops
    torch.manual_seed(5)
    x = (torch.randn((n, d, h, w, cin), device=gpu) * 0.8 + 0.2 + off).to(torch.bfloat16)
    dy = (torch.randn((n, d, h, w, cout), device=gpu) * 0.3).to(torch.bfloat16)
    wt = torch.randn((cout, cin, 3, 3, 3), device=gpu) * 0.05
    (pf, pd, st), = ops.wstd_fwd_batch([(wt, True, True)], torch.bfloat16)
    gn = (ops.gn_stats(x, groups), 1 + 0.1 * torch.randn(cin, device=gpu), 0.1 * torch.randn(cin, device=gpu), groups)
    return x, dy, pd, gn


def _separate(x, dy, pd, gn):
    from u3d import ops
    cin = x.shape[-1]
    da = ops.conv_dgrad(dy, pd, cin, tuple(x.shape[:4]), 3, 1)
    dg, db = torch.zeros(cin, device=x.device), torch.zeros(cin, device=x.device)
    dx = ops.gn_bwd(da, x, gn[0], gn[1], gn[2], gn[3], dgamma=dg, dbeta=db)
    return da, dx, dg, db


def _fused(x, dy, pd, gn, dx0=None):
    from u3d import ops
    cin = x.shape[-1]
    r = ops.conv_dgrad_gn(dy, pd, cin, x, 3, 1, gn)
    assert r is not None, "the fused brick path did not run"
    da, parts = r
    n, d, h, w = x.shape[:4]
    assert parts.shape[1] == ops.query("u3d_convg_brick_gn_nparts", n, cin, d, h, w, dy.shape[-1])
    dg, db = torch.zeros(cin, device=x.device), torch.zeros(cin, device=x.device)
    dx = ops.gn_bwd_parts(da, x, parts, gn[0], gn[1], gn[2], gn[3], dx=dx0, accumulate=dx0 is not None,
                          dgamma=dg, dbeta=db)
    return da, dx, dg, db, parts


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:4])) + f"_c{c[4]}-{c[5]}_g{c[6]}_o{c[7]:g}")
def test_fused_brick_gn_backward_matches_separate(gpu, case):
    x, dy, pd, gn = _setup(gpu, *case)
    a_da, a_dx, a_dg, a_db = _separate(x, dy, pd, gn)
    b_da, b_dx, b_dg, b_db, parts = _fused(x, dy, pd, gn)
    c_da, c_dx, c_dg, c_db, parts2 = _fused(x, dy, pd, gn)
    torch.cuda.synchronize()
    assert torch.equal(a_da, b_da)  # same schedule, same stores
    assert torch.equal(parts, parts2) and torch.equal(b_dx, c_dx) and torch.equal(b_dg, c_dg)  # deterministic
    for a, b, tol in ((a_dg, b_dg, 2e-5), (a_db, b_db, 2e-5)):
        err = ((a - b).norm() / a.norm().clamp_min(1e-12)).item()
        assert err < tol, err
    err = ((a_dx.float() - b_dx.float()).norm() / a_dx.float().norm()).item()
    assert err < 2e-3, err  # bf16 output: a coefficient ulp moves some roundings
    assert (a_dx != b_dx).float().mean().item() < 0.02


def test_fused_brick_gn_backward_vs_fp64(gpu):
    """The partial sums themselves against an fp64 restatement over the same bf16 dA and x (sum g, sum g*xhat)."""
    x, dy, pd, gn = _setup(gpu, 2, 24, 24, 24, 64, 64, 16, 40.0)
    from u3d import ops
    da, parts = ops.conv_dgrad_gn(dy, pd, 64, x, 3, 1, gn)
    st, ga, be, G = gn
    n, c = x.shape[0], x.shape[-1]
    xv = x.double().reshape(n, -1, c)
    mean = st[:, :, 0].double().repeat_interleave(c // G, dim=1)[:, None, :]
    rstd = st[:, :, 1].double().repeat_interleave(c // G, dim=1)[:, None, :]
    m = ((xv - mean) * rstd * ga.double() + be.double()) > 0
    g = torch.where(m, da.double().reshape(n, -1, c), torch.zeros((), dtype=torch.float64, device=gpu))
    ref = torch.stack([g.sum(1), (g * (xv - mean) * rstd).sum(1)], -1)  # [n][c][2]
    got = parts.double().sum(1)
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err


def test_fused_brick_gn_backward_accumulates(gpu):
    x, dy, pd, gn = _setup(gpu, 2, 24, 24, 24, 64, 64, 16, 0.0)
    _, a_dx, _, _ = _separate(x, dy, pd, gn)
    base = (torch.randn_like(x.float()) * 0.1).to(torch.bfloat16)
    _, b_dx, _, _, _ = _fused(x, dy, pd, gn, dx0=base.clone())
    ref = base.float() + a_dx.float()
    err = ((b_dx.float() - ref).norm() / ref.norm()).item()
    assert err < 4e-3, err
