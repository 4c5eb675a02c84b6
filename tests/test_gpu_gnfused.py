"""GroupNorm backward with its partial pass fused into the data-gradient ring's epilogue (ops.conv_dgrad_gn +
ops.gn_bwd_parts; u3d_conv32_ring_dgrad_gn + u3d_gn_bwd_parts) against the separate form (conv_dgrad + gn_bwd):
dA bitwise equal (the same ring, the same stores), dx / dgamma / dbeta equal up to fp32 reassociation of the
per-channel sums, and deterministic run to run. Reference: autograd of NoBottleneck's relu(gn(x)) -> conv3x3x3
(unet3D.py:44-73) — the backward of each gn1/gn2 at the 32-channel levels."""

import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # n, d, h, w, groups
    (2, 24, 24, 24, 16),
    (1, 13, 20, 37, 16),   # ragged tiles (partial 16x16 columns, depth not a multiple of anything)
    (2, 16, 16, 48, 8),    # 4 channels per group
    (2, 96, 96, 96, 16),   # the benchmark level
]


def _setup(gpu, n, d, h, w, groups):
    from u3d import ops
    torch.manual_seed(11)
    x = (torch.randn((n, d, h, w, 32), device=gpu) * 0.8 + 0.2).to(torch.bfloat16)
    dy = (torch.randn((n, d, h, w, 32), device=gpu) * 0.3).to(torch.bfloat16)
    wt = torch.randn((32, 32, 3, 3, 3), device=gpu) * 0.05
    (pf, pd, st), = ops.wstd_fwd_batch([(wt, True, True)], torch.bfloat16)
    gn = (ops.gn_stats(x, groups), 1 + 0.1 * torch.randn(32, device=gpu), 0.1 * torch.randn(32, device=gpu), groups)
    return x, dy, pd, gn


def _separate(x, dy, pd, gn):
    from u3d import ops
    da = ops.conv_dgrad(dy, pd, 32, tuple(x.shape[:4]), 3, 1)
    dg, db = torch.zeros(32, device=x.device), torch.zeros(32, device=x.device)
    dx = ops.gn_bwd(da, x, gn[0], gn[1], gn[2], gn[3], dgamma=dg, dbeta=db)
    return da, dx, dg, db


def _fused(x, dy, pd, gn, dx0=None):
    from u3d import ops
    r = ops.conv_dgrad_gn(dy, pd, 32, x, 3, 1, gn)
    assert r is not None, "the fused ring path did not run"
    da, parts = r
    dg, db = torch.zeros(32, device=x.device), torch.zeros(32, device=x.device)
    dx = ops.gn_bwd_parts(da, x, parts, gn[0], gn[1], gn[2], gn[3], dx=dx0, accumulate=dx0 is not None,
                          dgamma=dg, dbeta=db)
    return da, dx, dg, db, parts


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:4])) + f"_g{c[4]}")
def test_fused_gn_backward_matches_separate(gpu, case):
    x, dy, pd, gn = _setup(gpu, *case)
    a_da, a_dx, a_dg, a_db = _separate(x, dy, pd, gn)
    b_da, b_dx, b_dg, b_db, parts = _fused(x, dy, pd, gn)
    c_da, c_dx, c_dg, c_db, parts2 = _fused(x, dy, pd, gn)
    torch.cuda.synchronize()
    assert torch.equal(a_da, b_da)          # same ring, same stores
    assert torch.equal(parts, parts2) and torch.equal(b_dx, c_dx) and torch.equal(b_dg, c_dg)  # deterministic
    # fp32 per-workgroup sums vs the partial pass's per-block sums: reassociation only
    for a, b, tol in ((a_dg, b_dg, 2e-5), (a_db, b_db, 2e-5)):
        err = ((a - b).norm() / a.norm().clamp_min(1e-12)).item()
        assert err < tol, err
    err = ((a_dx.float() - b_dx.float()).norm() / a_dx.float().norm()).item()
    assert err < 2e-3, err  # bf16 output: a coefficient ulp moves some roundings
    mism = (a_dx != b_dx).float().mean().item()
    assert mism < 0.02, mism


def test_fused_gn_backward_accumulates(gpu):
    x, dy, pd, gn = _setup(gpu, 2, 20, 24, 32, 16)
    _, a_dx, _, _ = _separate(x, dy, pd, gn)
    base = (torch.randn_like(x.float()) * 0.1).to(torch.bfloat16)
    _, b_dx, _, _, _ = _fused(x, dy, pd, gn, dx0=base.clone())
    ref = (base.float() + a_dx.float())
    err = ((b_dx.float() - ref).norm() / ref.norm()).item()
    assert err < 4e-3, err


def test_fused_path_not_taken_under_collective(gpu):
    """While a bucket all-reduce is in flight the data-gradient ring runs its work-stealing form (per-sub-chunk
    claims): the fused epilogue is static-schedule only, so conv_dgrad_gn declines and the caller takes gn_bwd."""
    from u3d import ops
    x, dy, pd, gn = _setup(gpu, 1, 8, 16, 16, 16)
    ops.COLLECTIVE_IN_FLIGHT[0] = True
    try:
        assert ops.conv_dgrad_gn(dy, pd, 32, x, 3, 1, gn) is None
    finally:
        ops.COLLECTIVE_IN_FLIGHT[0] = False


@pytest.mark.parametrize("case", CASES[:3] + [(2, 96, 96, 96, 16)], ids=lambda c: "x".join(map(str, c[:4])) + f"_g{c[4]}")
def test_fused_finalize_in_ring(gpu, case, monkeypatch):
    """Round 5: the finalize in the ring launch (its last-arriving workgroup writes coef / dgamma / dbeta;
    u3d_conv32_ring_dgrad_gn_fused + u3d_gn_bwd_apply_coef) against the separate form: dA bitwise, dgamma / dbeta
    rel <= 2e-5, dx rel <= 2e-3; two runs bitwise equal (and the arrival counter left at zero)."""
    from u3d import ops
    monkeypatch.setattr(ops, "FUSED_FINALIZE", True)  # (an option, off by default)
    x, dy, pd, gn = _setup(gpu, *case)
    a_da, a_dx, a_dg, a_db = _separate(x, dy, pd, gn)
    outs = []
    for _ in range(2):
        dg, db = torch.full((32,), 5.0, device=gpu), torch.full((32,), 5.0, device=gpu)  # overwritten
        r = ops.conv_dgrad_gn(dy, pd, 32, x, 3, 1, gn, dgb=lambda: (dg, db))
        assert r is not None and isinstance(r[1], tuple) and r[1][0] == "coef", "the fused ring finalize did not run"
        dx = ops.gn_bwd_apply_coef(r[0], x, r[1][1], gn[3])
        outs.append((r[0], dx, dg, db, r[1][1]))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], a_da)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    _, dx, dg, db, _ = outs[0]
    for a, b in ((a_dg, dg), (a_db, db)):
        err = ((a - b).norm() / a.norm().clamp_min(1e-12)).item()
        assert err < 2e-5, err
    err = ((a_dx.float() - dx.float()).norm() / a_dx.float().norm()).item()
    assert err < 2e-3, err
