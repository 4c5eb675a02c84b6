"""GroupNorm(16) statistics taken in the epilogue of the producing kernel (round 5): the conv1 stem
(u3d_stem1_fwd_stats) and the decoder's trilinear x2 upsample + skip (u3d_upsample2x_add_stats). Their outputs must be
bitwise those of the statistics-free launches, and the statistics those of the separate pass (u3d_gn_stats: shifted
partial sums, fp64 combine) on the stored bf16 output: mean within 1e-4 of the output scale, rstd within 5e-4
relative (the tolerance of the ring conv's epilogue statistics, test_gpu_bf16.py). The epilogue forms sum unshifted fp32
values per block, so cases with |mean| / std ~ 3-10 are included; ragged rows (w * c / 8 not a multiple of the block),
every channel count of the trunk's decoder (c / 16 = 2, 4, 8, 16 channels per group), n = 1 and n = 3.
Reference: GroupNorm in NoBottleneck (unet3D.py:44-53) after conv1 (:1632) and after upsamplex2 + skip (:1764-1783)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(s16, ref, y):
    scale = y.float().abs().max().item()
    dm = (s16[..., 0] - ref[..., 0]).abs().max().item()
    dr = ((s16[..., 1] - ref[..., 1]).abs() / ref[..., 1]).max().item()
    print(f"mean err {dm / scale:.2e} of scale, rstd rel err {dr:.2e}")
    assert dm < 1e-4 * scale
    assert dr < 5e-4


@pytest.mark.parametrize("n,dims,off", [(2, (16, 16, 16), 0.0), (1, (8, 16, 32), 3.0), (3, (4, 8, 24), -2.0),
                                        (2, (32, 32, 32), 0.5)])
def test_stem1_epilogue_stats(gpu, n, dims, off):
    from u3d import ops
    torch.manual_seed(11)
    x = torch.randn((n, 1) + dims, device=gpu) + off
    w = torch.randn(32, 1, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    y, s16 = ops.stem_fwd_stats(x, pf, 32, 1, torch.bfloat16)
    assert s16 is not None
    y2 = ops.stem_fwd(x, pf, 32, 1, torch.bfloat16)
    assert torch.equal(y, y2)
    _close(s16, ops.gn_stats(y, 16), y)


def test_stem1_stats_unsupported_shape_falls_back(gpu):
    """d*h*w not a multiple of 256: no epilogue form (blocks would straddle samples); the caller takes the pass."""
    from u3d import _lib, ops
    assert _lib.query("u3d_stem1_stats_ws_floats", 2, 5, 7, 9) == 0
    x = torch.randn((2, 1, 5, 7, 9), device=gpu)
    pf, _, _ = ops.wstd_fwd(torch.randn(32, 1, 3, 3, 3, device=gpu), torch.bfloat16, True, need_dgrad=False)
    y, s16 = ops.stem_fwd_stats(x, pf, 32, 1, torch.bfloat16)
    assert s16 is None and y.shape == (2, 5, 7, 9, 32)


@pytest.mark.parametrize("n,c,dims,skip,off", [
    (2, 32, (8, 12, 48), True, 0.0),     # 96^3-level channel count; w * c / 8 = 192: one partial block per row
    (2, 64, (6, 10, 24), True, 4.0),     # 48^3 level
    (1, 128, (5, 6, 12), True, -3.0),    # 24^3 level
    (3, 256, (3, 3, 6), True, 1.0),      # 12^3 level: 16 channels per group, two chunks per group
    (2, 32, (4, 4, 100), False, 10.0),   # ragged: 400 (iw, chunk) pairs -> a full and a partial block per row
    (2, 64, (24, 24, 24), True, 0.3),    # bench-like 2 x 24^3 x 64 -> 48^3
])
def test_upsample_epilogue_stats(gpu, n, c, dims, skip, off):
    from u3d import ops
    torch.manual_seed(12)
    x = (torch.randn((n,) + dims + (c,), device=gpu) * 2 + off).to(torch.bfloat16)
    sk = (torch.randn((n,) + tuple(2 * d for d in dims) + (c,), device=gpu) + 0.5 * off).to(torch.bfloat16) \
        if skip else None
    y, s16 = ops.upsample2x_add_stats(x, sk)
    assert s16 is not None
    y2 = ops.upsample2x_add(x, sk)
    assert torch.equal(y, y2)
    _close(s16, ops.gn_stats(y, 16), y)


@pytest.mark.parametrize("n,cin,cout,dims,res,flip", [
    (2, 256, 256, (12, 12, 12), True, False),   # layer3 / x8_resb blocks (nks 4)
    (2, 256, 256, (6, 6, 6), False, False),     # layer4 (nks 8)
    (1, 128, 128, (12, 12, 12), True, False),
    (3, 64, 64, (8, 8, 8), True, False),        # n = 3, 64 channels (4 per group)
    (2, 256, 128, (12, 12, 12), False, True),   # data gradient (flip): combine only
    (2, 256, 256, (6, 6, 6), False, True),
])
def test_conv_small_in_kernel_combine(gpu, n, cin, cout, dims, res, flip):
    """u3d_conv_small2: the split-K slabs combined by each output tile's last-arriving workgroup inside the conv launch
    give bitwise the output of the two-kernel form (u3d_conv_small + small_reduce_kernel: same slab order), and the
    forward's output GroupNorm(16) statistics from that combine match the statistics pass. Two launches in a row check
    that the arrival counters were left at zero."""
    from u3d import ops
    torch.manual_seed(13)
    x = (torch.randn((n,) + dims + (cin,), device=gpu) + 0.7).to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    G = 16
    gn = None if flip else (ops.gn_stats(x, G), 1 + 0.1 * torch.randn(cin, device=gpu), 0.1 * torch.randn(cin, device=gpu),
                            G)
    r = (torch.randn((n,) + dims + (cout,), device=gpu) * 3 + 2).to(torch.bfloat16) if res else None
    pk, co = pf, cout  # ([27][cout_p][cin_p]: the layout both directions read; fused vs two-kernel on the same pack)
    assert ops._use_small(torch.bfloat16, cin, cout, 3, 1, (n,) + dims)
    outs = []
    for fuse in (False, True, True):
        ops.SMALL_FUSE, old = fuse, ops.SMALL_FUSE
        try:
            y = torch.empty((n,) + dims + (co,), dtype=torch.bfloat16, device=gpu)
            st = ops.conv_small(1 if flip else 0, x, cin, pk, co, gn, r, y, want_stats=not flip)
        finally:
            ops.SMALL_FUSE = old
        outs.append((y, st))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[1][0], outs[2][0])
    if not flip:
        assert outs[0][1] is None and outs[1][1] is not None
        assert torch.equal(outs[1][1], outs[2][1])
        _close(outs[1][1], ops.gn_stats(outs[1][0], 16), outs[1][0])


@pytest.mark.parametrize("kind,n,c,dims,res", [
    ("ring", 2, 32, (24, 24, 24), True),    # 32 -> 32 ring conv (the 96^3 level's kernel), 2 samples
    ("ring", 1, 32, (10, 16, 40), False),
    ("ring", 3, 32, (9, 12, 16), True),
    ("brick", 2, 64, (24, 24, 24), True),   # persistent brick (48^3 / 24^3 levels)
    ("brick", 2, 128, (16, 24, 32), False),
    ("brick", 3, 64, (16, 32, 32), True),
])
def test_fused_finalize_matches_finalize_kernel(gpu, monkeypatch, kind, n, c, dims, res):
    """The ring / persistent-brick epilogue statistics finalized by the conv launch's last-arriving workgroup
    (ops.FUSED_FINALIZE, round 5) against the separate finalize kernel on the same partials: outputs bitwise equal,
    statistics equal up to the fp64 combine order (<= 1e-6 relative), and two fused launches in a row bitwise equal
    (the arrival counter is left at zero)."""
    from u3d import ops
    torch.manual_seed(17)
    x = (torch.randn((n,) + dims + (c,), device=gpu) + 0.4).to(torch.bfloat16)
    w = torch.randn(c, c, 3, 3, 3, device=gpu) * 0.1
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    gn = (ops.gn_stats(x, 16), 1 + 0.1 * torch.randn(c, device=gpu), 0.1 * torch.randn(c, device=gpu), 16)
    r = (torch.randn((n,) + dims + (c,), device=gpu) + 1).to(torch.bfloat16) if res else None
    if kind == "ring":
        assert ops._use_conv32(torch.bfloat16, c, c, 3, 1, n, dims[2])
    else:
        assert ops._use_gen_brick(torch.bfloat16, c, c, 3, 1, (n,) + dims)
    outs = []
    for fused in (False, True, True):
        monkeypatch.setattr(ops, "FUSED_FINALIZE", fused)
        y, st = ops.conv_fwd_stats(x, pf, c, 3, 1, gn, residual=r)
        assert st is not None
        outs.append((y, st))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[1][0], outs[2][0]) and torch.equal(outs[1][1], outs[2][1])
    rel = ((outs[1][1] - outs[0][1]).abs() / outs[0][1].abs().clamp_min(1e-6)).max().item()
    assert rel <= 1e-6, rel
