"""bf16 kernel paths (the bench precision) against an fp64 CPU reference computed on the SAME bf16-rounded
operands, so the only differences are fp32 accumulation order and the final bf16 rounding of outputs.
Tolerances: outputs rounded to bf16 -> 1e-2 of the tensor's max |value|; fp32 partial sums (weight grads)
-> 2e-3 of max."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).double()


def _case(gpu, n, cin, cout, dims, gn, seed):
    from u3d import ops
    torch.manual_seed(seed)
    x = (torch.randn((n,) + dims + (cin,), device=gpu) * 1.5 + 0.3).to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, 3, device=gpu)
    G = 16 if cin % 16 == 0 else 8
    st = ops.gn_stats(x, G) if gn else None
    ga = (1 + 0.1 * torch.randn(cin, device=gpu))
    be = 0.1 * torch.randn(cin, device=gpu)
    return x, w, st, ga, be, G


def _act_ref(x, st, ga, be, G):
    """A = relu(x*sc + sh) in fp32 exactly as the kernel prologue, rounded to bf16."""
    xf = x.float().cpu()
    if st is None:
        return xf.double()
    n, c = xf.shape[0], xf.shape[-1]
    s = st.cpu()
    g = torch.arange(c) // (c // G)
    mean, rstd = s[:, g, 0], s[:, g, 1]               # [n, c]
    sc = rstd * ga.cpu()[None]
    sh = be.cpu()[None] - mean * sc
    a = torch.clamp_min(torch.addcmul(sh.view(n, 1, 1, 1, c), xf, sc.view(n, 1, 1, 1, c)), 0)
    return _bf(a)


SHAPES = [(2, 32, 32, (12, 10, 16), 1), (1, 32, 32, (5, 9, 70), 1), (1, 32, 64, (8, 12, 18), 2), (2, 64, 64, (6, 8, 9), 1),
          (1, 64, 32, (10, 6, 8), 1), (2, 128, 128, (4, 4, 4), 1), (1, 24, 24, (7, 9, 11), 1),
          (2, 32, 32, (4, 10, 64), 1), (1, 32, 32, (3, 8, 32), 1), (1, 64, 128, (6, 9, 20), 1),
          (2, 32, 32, (6, 7, 96), 1), (3, 32, 32, (9, 5, 32), 1),
          (2, 32, 64, (12, 16, 34), 2), (1, 64, 128, (8, 8, 8), 2), (2, 128, 256, (12, 12, 12), 2),
          (1, 256, 256, (6, 6, 6), 2), (1, 40, 48, (6, 10, 14), 2)]


@pytest.fixture(params=["auto", "gen_brick", "igemm", "small", "ring", "brick32"])
def conv_path(request):
    """auto = production routing; gen_brick = force the generic halo-brick kernel; igemm = force implicit GEMM."""
    from u3d import ops
    saved = (ops.BRICK_MIN_WG, ops.USE_CONV32_BRICK, ops.USE_GEN_BRICK, ops.USE_S2_BRICK, ops.USE_SMALL_CONV,
             ops.SMALL_MAX_VOX, ops.CONV32_FN)
    if request.param == "gen_brick":
        ops.BRICK_MIN_WG, ops.USE_CONV32_BRICK, ops.USE_SMALL_CONV = 0, False, False
    elif request.param == "igemm":
        ops.USE_CONV32_BRICK, ops.USE_GEN_BRICK, ops.USE_S2_BRICK, ops.USE_SMALL_CONV = False, False, False, False
    elif request.param == "small":
        ops.USE_CONV32_BRICK, ops.SMALL_MAX_VOX = False, 1 << 40
    elif request.param == "ring":
        ops.CONV32_FN, ops.USE_SMALL_CONV = "u3d_conv32_ring", False
    elif request.param == "brick32":
        ops.CONV32_FN, ops.USE_SMALL_CONV = "u3d_conv32_brick", False
    yield request.param
    (ops.BRICK_MIN_WG, ops.USE_CONV32_BRICK, ops.USE_GEN_BRICK, ops.USE_S2_BRICK, ops.USE_SMALL_CONV,
     ops.SMALL_MAX_VOX, ops.CONV32_FN) = saved


@pytest.mark.parametrize("n,cin,cout,dims,s", SHAPES)
def test_bf16_conv_fwd(gpu, conv_path, n, cin, cout, dims, s):
    from u3d import ops
    x, w, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 1)
    pf, pd, wst = ops.wstd_fwd(w, torch.bfloat16, True)
    od = tuple(ops.out_dim(d, 3, s) for d in dims)
    res = torch.randn((n,) + od + (cout,), device=gpu).to(torch.bfloat16)
    y = ops.conv_fwd(x, pf, cout, 3, s, (st, ga, be, G), residual=res)
    a = _act_ref(x, st, ga, be, G).permute(0, 4, 1, 2, 3)
    wq = pf.float().cpu()[:, :cout, :cin].permute(1, 2, 0).reshape(cout, cin, 3, 3, 3).double()
    ref = F.conv3d(a, wq, stride=s, padding=1).permute(0, 2, 3, 4, 1) + res.double().cpu()
    err = (y.double().cpu() - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("n,cin,cout,dims,s", SHAPES)
def test_bf16_conv_dgrad(gpu, conv_path, n, cin, cout, dims, s):
    from u3d import ops
    if s == 2 and any(d % 2 for d in dims) and conv_path == "igemm":
        pytest.skip("the parity-class implicit-GEMM stride-2 dgrad needs even dims (as the trunk has)")
    x, w, *_ = _case(gpu, n, cin, cout, dims, False, 2)
    pf, pd, wst = ops.wstd_fwd(w, torch.bfloat16, True)
    od = tuple(ops.out_dim(d, 3, s) for d in dims)
    dy = torch.randn((n,) + od + (cout,), device=gpu).to(torch.bfloat16)
    dx = ops.conv_dgrad(dy, pd, cin, (n,) + dims, 3, s)
    wq = pf.float().cpu()[:, :cout, :cin].permute(1, 2, 0).reshape(cout, cin, 3, 3, 3).double()
    ref = torch.nn.grad.conv3d_input((n, cin) + dims, wq, _bf(dy.cpu().float()).permute(0, 4, 1, 2, 3),
                                     stride=s, padding=1).permute(0, 2, 3, 4, 1)
    err = (dx.double().cpu() - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("brick", ["ring", True, False])
@pytest.mark.parametrize("n,cin,cout,dims,s", SHAPES)
def test_bf16_conv_wgrad(gpu, n, cin, cout, dims, s, brick):
    from u3d import ops
    if brick == "ring" and s != 1:
        pytest.skip("the ring weight gradient serves stride 1")
    x, w, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 3)
    od = tuple(ops.out_dim(d, 3, s) for d in dims)
    dy = torch.randn((n,) + od + (cout,), device=gpu).to(torch.bfloat16)
    part, ns = ops.conv_wgrad(dy, x, 3, s, (st, ga, be, G), brick=brick)
    dw = part.sum(0).cpu().double()[:, :cout, :cin]                       # [27, cout, cin]
    a = _act_ref(x, st, ga, be, G).permute(0, 4, 1, 2, 3)
    ref = torch.nn.grad.conv3d_weight(a, (cout, cin, 3, 3, 3), _bf(dy.cpu().float()).permute(0, 4, 1, 2, 3),
                                      stride=s, padding=1)
    ref = ref.reshape(cout, cin, 27).permute(2, 0, 1)
    err = (dw - ref).abs().max().item()
    assert err < 2e-3 * ref.abs().max().item(), err


@pytest.mark.parametrize("n,cin,cout,dims", [(1, 32, 64, (8, 12, 18)), (2, 64, 128, (12, 10, 16)), (3, 40, 48, (9, 10, 14)),
                                             (2, 32, 64, (96, 96, 96)), (3, 32, 64, (13, 17, 20))])
def test_wgrad_brick_s2_three_plane_bricks_match_two(gpu, n, cin, cout, dims):
    """Stride-2 brick weight gradient with 3-plane output bricks (round 6 default, OPT WB_S2BD = 3) against 2-plane
    bricks: the same products over other brick and split boundaries (samples change inside a split: the GroupNorm
    coefficients staged in LDS are refreshed), so equal up to the fp32 order of the sums: <= 1e-5 of max |dW|; both
    against the fp64 reference within the bf16 bound of test_bf16_conv_wgrad."""
    from u3d import ops
    x, w, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 11)
    od = tuple(ops.out_dim(d, 3, 2) for d in dims)
    dy = torch.randn((n,) + od + (cout,), device=gpu).to(torch.bfloat16)
    with ops.option("WB_S2BD", 3):
        part3, _ = ops.conv_wgrad(dy, x, 3, 2, (st, ga, be, G), brick=True)
    with ops.option("WB_S2BD", 2):
        part2, _ = ops.conv_wgrad(dy, x, 3, 2, (st, ga, be, G), brick=True)
    a, b = part3.double().sum(0), part2.double().sum(0)
    scale = b.abs().max().item()
    assert (a - b).abs().max().item() <= 1e-5 * scale
    if dims[0] <= 16:
        a_ref = _act_ref(x, st, ga, be, G).permute(0, 4, 1, 2, 3)
        ref = torch.nn.grad.conv3d_weight(a_ref, (cout, cin, 3, 3, 3), _bf(dy.cpu().float()).permute(0, 4, 1, 2, 3),
                                          stride=2, padding=1).reshape(cout, cin, 27).permute(2, 0, 1)
        err = (a.cpu()[:, :cout, :cin] - ref).abs().max().item()
        assert err < 2e-3 * ref.abs().max().item(), err


@pytest.mark.parametrize("n,cin,cout,dims", [(1, 32, 64, (8, 12, 18)), (2, 64, 128, (12, 10, 16)), (1, 40, 48, (6, 10, 14))])
def test_wgrad_brick_s2_two_co_tiles_matches_one(gpu, n, cin, cout, dims):
    """Stride-2 brick weight gradient with two 32-wide co tiles per workgroup (one staged halo for 64 output channels,
    the default) against one co tile per workgroup (OPT WB_S2CO64 = 0): each output element is the same MFMA chain
    over the same bricks; only the split boundaries (the split count follows the workgroup count) and so the fp32
    order of the split sums differ: <= 1e-5 of max |dW|."""
    from u3d import ops
    x, w, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 7)
    od = tuple(ops.out_dim(d, 3, 2) for d in dims)
    dy = torch.randn((n,) + od + (cout,), device=gpu).to(torch.bfloat16)
    part, _ = ops.conv_wgrad(dy, x, 3, 2, (st, ga, be, G), brick=True)
    with ops.option("WB_S2CO64", 0):
        part1, _ = ops.conv_wgrad(dy, x, 3, 2, (st, ga, be, G), brick=True)
    a, b = part.double().sum(0), part1.double().sum(0)
    assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item()


def test_bf16_gn_bwd_and_upsample(gpu):
    from u3d import ops
    torch.manual_seed(4)
    x = (torch.randn(2, 6, 8, 10, 64, device=gpu) * 2 + 1).to(torch.bfloat16)
    st = ops.gn_stats(x, 16)
    ref_st = x.float().cpu().reshape(2, -1, 16, 4).permute(0, 2, 1, 3).reshape(2, 16, -1)
    assert (st[..., 0].cpu() - ref_st.mean(-1)).abs().max() < 1e-5
    assert ((st[..., 1].cpu() - ref_st.var(-1, unbiased=False).add(1e-5).rsqrt()).abs()
            / st[..., 1].cpu()).max() < 1e-5
    y = ops.upsample2x_add(x)
    ref = F.interpolate(x.float().cpu().permute(0, 4, 1, 2, 3), scale_factor=2, mode="trilinear")
    assert (y.float().cpu().permute(0, 4, 1, 2, 3) - ref).abs().max() < 1e-2 * ref.abs().max()


def test_wstd_batch_matches_single(gpu):
    """Batched weight standardisation (one launch for every conv) == the per-conv kernels."""
    from u3d import ops
    torch.manual_seed(5)
    shapes = [(32, 1, 3, True), (32, 32, 3, True), (64, 32, 3, True), (64, 32, 1, True), (320, 256, 3, True),
              (8, 32, 1, False), (24, 40, 3, True)]
    ws = [torch.randn(co, ci, k, k, k, device=gpu) * 0.1 + 0.01 for co, ci, k, _ in shapes]
    for dt in (torch.float32, torch.bfloat16):
        outs = ops.wstd_fwd_batch([(w, std, ci > 4) for w, (co, ci, k, std) in zip(ws, shapes)], dt)
        for w, (co, ci, k, std), (pf, pd, st) in zip(ws, shapes, outs):
            pf1, pd1, st1 = ops.wstd_fwd(w, dt, std, need_dgrad=ci > 4)
            tol = 1e-6 if dt == torch.float32 else 1e-2
            assert (pf.float() - pf1.float()).abs().max().item() <= tol * pf1.float().abs().max().item()
            if pd1 is not None:
                assert torch.equal(pd.float().permute(0, 2, 1), pf.float())
            if std:
                assert torch.allclose(st, st1, rtol=1e-6, atol=1e-7)
    # backward: random split slabs, nsplit 1 / 3 / 37
    items, refs = [], []
    for (w, (co, ci, k, std)), ns in zip(zip(ws, shapes), [1, 3, 37, 2, 5, 1, 4]):
        _, _, st = ops.wstd_fwd(w, torch.float32, std, need_dgrad=False)
        part = torch.randn((ns, k ** 3, ops.round32(co), ops.round32(ci)), device=gpu)
        ref = ops.wstd_bwd(part.clone(), ns, w, st, std)
        dw = torch.empty_like(w)
        items.append((part, ns, w, st, std, dw, False))
        refs.append(ref)
    ops.wstd_bwd_batch(items)
    for (part, ns, w, st, std, dw, _), ref in zip(items, refs):
        assert (dw - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_wstd_bwd_row_kernel_matches_chunked(gpu):
    """Weight-standardisation backward, one row per block from registers (WSTD_ROW=1, round 4) == the chunked LDS
    kernel (WSTD_ROW=0): the same per-row sums in another fp32 order (rows up to 56 x 256 long), accumulate on/off."""
    from u3d import ops
    torch.manual_seed(9)
    shapes = [(32, 1, 3, True), (32, 32, 3, True), (64, 64, 1, True), (256, 256, 3, True), (48, 512, 3, True),
              (8, 32, 1, False), (24, 40, 3, True)]
    ws = [torch.randn(co, ci, k, k, k, device=gpu) * 0.1 + 0.02 for co, ci, k, _ in shapes]
    sts = [ops.wstd_fwd(w, torch.float32, std, need_dgrad=False)[2] for w, (_, _, _, std) in zip(ws, shapes)]
    parts = [torch.randn((ns, k ** 3, ops.round32(co), ops.round32(ci)), device=gpu)
             for (co, ci, k, _), ns in zip(shapes, [1, 3, 4, 9, 2, 1, 5])]
    base = [torch.randn_like(w) for w in ws]
    out = {}
    for row in (0, 1):
        for acc in (False, True):
            dws = [b.clone() for b in base]
            items = [(p.clone(), p.shape[0], w, st, std, dw, acc)
                     for p, w, st, (_, _, _, std), dw in zip(parts, ws, sts, shapes, dws)]
            with ops.option("WSTD_ROW", row):
                ops.wstd_bwd_batch(items)
            out[row, acc] = dws
    for acc in (False, True):
        for a, b in zip(out[0, acc], out[1, acc]):
            assert (a - b).abs().max().item() <= 2e-6 * a.abs().max().item()


@pytest.mark.parametrize("n,cin,cout,dims,s", [(2, 32, 16, (8, 10, 12), 1), (2, 32, 64, (8, 10, 12), 2),
                                               (1, 64, 128, (6, 6, 7), 2), (2, 320, 320, (3, 3, 3), 1),
                                               (1, 32, 8, (5, 7, 9), 1), (2, 32, 32, (40, 40, 40), 2)])
def test_bf16_conv_wgrad_1x1(gpu, n, cin, cout, dims, s):
    """1^3 weight gradient kernel (downsample / heads), GN prologue, strides 1 and 2."""
    from u3d import ops
    x, w, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 6)
    od = tuple(ops.out_dim(d, 1, s) for d in dims)
    dy = torch.randn((n,) + od + (cout,), device=gpu).to(torch.bfloat16)
    part, ns = ops.conv_wgrad(dy, x, 1, s, (st, ga, be, G))
    dw = part.sum(0).cpu().double()[0, :cout, :cin]
    a = _act_ref(x, st, ga, be, G).permute(0, 4, 1, 2, 3)
    ref = torch.nn.grad.conv3d_weight(a, (cout, cin, 1, 1, 1), _bf(dy.cpu().float()).permute(0, 4, 1, 2, 3),
                                      stride=s, padding=0)[:, :, 0, 0, 0]
    err = (dw - ref).abs().max().item()
    assert err < 2e-3 * ref.abs().max().item(), err


@pytest.mark.parametrize("dims", [(6, 10, 64), (3, 9, 32), (5, 7, 20), (33, 48, 64), (48, 64, 96), (35, 64, 96),
                                  (96, 96, 96)])
def test_bf16_stem_wgrad(gpu, dims):
    """conv1 (1 -> 32, 3^3, stride 1) weight gradient: MFMA kernel (w % 32 == 0) and the VALU kernel. The large
    volumes give the MFMA kernel's workgroups 1-7 bricks of 4 x 8 x 32 voxels each (its register prefetch of the next
    brick, partial last d bricks at d = 33 and 35); 96^3 is the bench's conv1."""
    from u3d import ops
    torch.manual_seed(7)
    n = 2
    x = torch.randn((n, 1) + dims, device=gpu)
    dy = torch.randn((n,) + dims + (32,), device=gpu).to(torch.bfloat16)
    part, ns = ops.stem_wgrad(dy, x, 1)
    dw = part.sum(0).cpu().double()[:, :32, 0]                            # [27, 32]
    xq = x.cpu().to(torch.bfloat16).double() if dims[2] % 32 == 0 else x.cpu().double()
    ref = torch.nn.grad.conv3d_weight(xq, (32, 1, 3, 3, 3), _bf(dy.cpu().float()).permute(0, 4, 1, 2, 3), padding=1)
    ref = ref.reshape(32, 27).t()
    err = (dw - ref).abs().max().item()
    assert err < 2e-3 * ref.abs().max().item(), err
    assert part[:, :, :, 1:].abs().max().item() == 0.0   # padded ci columns stay zero


@pytest.mark.parametrize("cin,cout,dims", [(32, 16, (6, 10, 12)), (32, 2, (4, 4, 7)), (64, 8, (3, 5, 6)),
                                           (16, 32, (2, 3, 4))])
def test_head_fwd_bwd(gpu, cin, cout, dims):
    """Streaming precls head (head.hip): logits = conv1(relu(gn(x))) + b; dA = dy W, bf16 dy, bias grad."""
    from u3d import ops
    n = 2
    x, _, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 7)
    w = torch.randn(cout, cin, 1, 1, 1, device=gpu)
    pf, pd, _ = ops.wstd_fwd(w, torch.bfloat16, False)
    b = torch.randn(cout, device=gpu)
    y = ops.head_fwd(x, pf, cout, b, (st, ga, be, G))
    a = _act_ref(x, st, ga, be, G)                                       # [n, ..., cin] fp64 of bf16 values
    wq = pf.float().cpu()[0, :cout, :cin].double()
    ref = a @ wq.t() + b.double().cpu()
    assert y.dtype == torch.float32
    assert (y.double().cpu() - ref).abs().max().item() < 1e-4 * ref.abs().max().item() + 1e-5
    dy = torch.randn(y.shape, device=gpu)
    db = torch.empty(cout, device=gpu)
    dA, dyb = ops.head_bwd(dy, pd, cin, dbias=db)
    dyq = _bf(dy.cpu())
    refA = dyq @ wq
    assert (dA.double().cpu() - refA).abs().max().item() < 1e-2 * refA.abs().max().item()
    assert torch.equal(dyb[..., :cout].cpu(), dy.to(torch.bfloat16).cpu())
    torch.testing.assert_close(db.cpu().double(), dy.cpu().double().reshape(-1, cout).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("cin,cout,dims,s", [(1, 32, (8, 10, 12), 1), (2, 24, (8, 6, 10), 2), (1, 8, (5, 7, 9), 1),
                                             (2, 32, (4, 4, 6), 1), (1, 32, (6, 9, 70), 1), (1, 32, (3, 4, 33), 1)])
def test_bf16_stem_fwd(gpu, cin, cout, dims, s):
    """Stem conv (fp32 input, bf16 packed weights, bf16 output; conv1 1 -> 32 on the packed-FMA kernel, the others on
    the generic kernel, all fp32 VALU math) against fp64 on the fp32 input."""
    from u3d import ops
    torch.manual_seed(3)
    x = torch.randn((2, cin) + dims, device=gpu)
    w = torch.randn(cout, cin, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    y = ops.stem_fwd(x, pf, cout, s, torch.bfloat16)
    wq = pf.float().cpu()[:, :cout, :cin].permute(1, 2, 0).reshape(cout, cin, 3, 3, 3).double()
    ref = F.conv3d(x.cpu().double(), wq, stride=s, padding=1).permute(0, 2, 3, 4, 1)
    err = (y.double().cpu() - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,cin,cout,dims", [(2, 32, 64, (8, 6, 10)), (1, 64, 128, (4, 4, 4)), (2, 256, 256, (4, 6, 2))])
def test_conv1_s2_dgrad_writes_every_voxel(gpu, dt, n, cin, cout, dims):
    """1^3 stride-2 data gradient (downsample convs): the odd-parity voxels get exact zeros from the GEMM kernel
    itself (no memset) — dx is pre-filled with NaN to prove every voxel is written."""
    from u3d import ops
    torch.manual_seed(4)
    w = torch.randn(cout, cin, 1, 1, 1, device=gpu)
    pf, pd, _ = ops.wstd_fwd(w, dt, True)
    od = tuple(ops.out_dim(d, 1, 2) for d in dims)
    dy = torch.randn((n,) + od + (cout,), device=gpu).to(dt)
    torch.cuda.synchronize()
    dx = ops.conv_dgrad(dy, pd, cin, (n,) + dims, 1, 2)
    wq = pf.float().cpu()[:, :cout, :cin].permute(1, 2, 0).reshape(cout, cin, 1, 1, 1).double()
    ref = torch.nn.grad.conv3d_input((n, cin) + dims, wq, dy.cpu().double().permute(0, 4, 1, 2, 3),
                                     stride=2).permute(0, 2, 3, 4, 1)
    got = dx.double().cpu()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() < 1e-2 * ref.abs().max().item()
    assert torch.count_nonzero(got[:, 1::2]) == 0 and torch.count_nonzero(got[:, :, 1::2]) == 0


@pytest.mark.parametrize("n,dims,res", [(2, (12, 10, 16), True), (1, (5, 9, 70), False), (3, (9, 5, 32), True),
                                        (2, (24, 24, 24), False)])
def test_ring_epilogue_gn_stats_match_stats_pass(gpu, n, dims, res):
    """The ring conv's epilogue-accumulated GroupNorm(16, 32) statistics (of the fp32 values just before the final
    bf16 rounding) equal the separate statistics pass (u3d_gn_stats, shifted fp64 combine) on the stored bf16 output:
    mean within 1e-4 of the output scale, rstd within 5e-4 relative (measured 1.1e-4)."""
    from u3d import ops
    x, w, st, ga, be, G = _case(gpu, n, 32, 32, dims, True, 7)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True)
    r = (torch.randn((n,) + dims + (32,), device=gpu) + 0.5).to(torch.bfloat16) if res else None
    y, s16 = ops.conv_fwd_stats(x, pf, 32, 3, 1, (st, ga, be, G), residual=r)
    assert s16 is not None
    y2 = ops.conv_fwd(x, pf, 32, 3, 1, (st, ga, be, G), residual=r)
    assert torch.equal(y, y2)                      # same output as the statistics-free launch
    ref = ops.gn_stats(y, 16)
    scale = y.float().abs().max().item()
    assert (s16[..., 0] - ref[..., 0]).abs().max().item() < 1e-4 * scale
    assert ((s16[..., 1] - ref[..., 1]).abs() / ref[..., 1]).max().item() < 5e-4


@pytest.mark.parametrize("dims", [(5, 7, 16), (3, 9, 20), (4, 4, 6)])
def test_stem_fwd_fp32_packed_kernel(gpu, dims):
    """cin=1 stride-1 32-channel stem: the packed one-voxel-per-lane kernel (any w, here 16, 20 and 6) against fp64 on
    the same fp32 operands."""
    from u3d import ops
    torch.manual_seed(4)
    x = torch.randn((2, 1) + dims, device=gpu)
    w = torch.randn(32, 1, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.float32, True, need_dgrad=False)
    y = ops.stem_fwd(x, pf, 32, 1, torch.float32)
    wq = pf.cpu()[:, :32, :1].permute(1, 2, 0).reshape(32, 1, 3, 3, 3).double()
    ref = F.conv3d(x.cpu().double(), wq, padding=1).permute(0, 2, 3, 4, 1)
    assert (y.double().cpu() - ref).abs().max().item() < 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("dims", [(5, 7, 16), (96, 96, 96)])
def test_stem1_packed_kernel_bitwise_equals_generic(gpu, dt, dims):
    """conv1 (cin 1 -> 32, stride 1): the packed-FMA kernel (scalar-loaded weights, v_pk_fma_f32) runs the same fp32 FMA
    chain per output as the generic kernel (OPT STEM1 = 0), so the outputs are bitwise equal."""
    from u3d import ops
    torch.manual_seed(6)
    x = torch.randn((2, 1) + dims, device=gpu)
    w = torch.randn(32, 1, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, dt, True, need_dgrad=False)
    with ops.option("STEM_MFMA", 0):  # (bf16 runs the matrix-core kernel by default: test_stem1_mfma_*)
        y = ops.stem_fwd(x, pf, 32, 1, dt)
    with ops.option("STEM1", 0):
        y0 = ops.stem_fwd(x, pf, 32, 1, dt)
    assert torch.equal(y, y0)


def _stem_ref_bf16_operands(x, pf):
    """fp64 conv1 on the operands the matrix-core kernel multiplies: the input and the packed weights in bf16."""
    wq = pf.float().cpu()[:, :32, :1].permute(1, 2, 0).reshape(32, 1, 3, 3, 3).double()
    return wq, x.to(torch.bfloat16).double().cpu()


@pytest.mark.parametrize("n,dims", [(2, (5, 7, 16)), (1, (3, 5, 7)), (2, (8, 8, 16)), (3, (4, 9, 33))])
def test_stem1_mfma_vs_fp64(gpu, n, dims):
    """bf16 conv1 (1 -> 32) on the matrix cores (round 6, stem1_mfma_kernel): bf16 operands (the reference's autocast
    conv1), exact products, fp32 sums: every output within one bf16 rounding of the fp64 conv on the same operands
    (+ 1e-6 of the largest output for the fp32 summation order); ragged voxel counts (partial waves) included."""
    from u3d import ops
    torch.manual_seed(21)
    x = torch.randn((n, 1) + dims, device=gpu) * 1.5 + 0.3
    w = torch.randn(32, 1, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    y = ops.stem_fwd(x, pf, 32, 1, torch.bfloat16)
    wq, xb = _stem_ref_bf16_operands(x, pf)
    ref = F.conv3d(xb, wq, padding=1).permute(0, 2, 3, 4, 1)
    d = (y.double().cpu() - ref).abs()
    assert bool((d <= ref.abs() * 2.0 ** -8 + 1e-6 * ref.abs().max()).all()), d.max().item()


def test_stem1_mfma_bench_size(gpu):
    """the bench's conv1 (2 x 96^3, with the epilogue statistics): sampled planes within one bf16 rounding of the fp64
    conv on the bf16 operands; the statistics form writes the same output as the plain form."""
    from u3d import ops
    torch.manual_seed(22)
    x = torch.rand((2, 1, 96, 96, 96), device=gpu) * 2 - 1
    w = torch.randn(32, 1, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    y, s16 = ops.stem_fwd_stats(x, pf, 32, 1, torch.bfloat16)
    assert s16 is not None
    assert torch.equal(y, ops.stem_fwd(x, pf, 32, 1, torch.bfloat16))
    wq, xb = _stem_ref_bf16_operands(x, pf)
    for n in range(2):
        for z in (0, 47, 95):
            lo, hi = max(0, z - 1), min(96, z + 2)
            ref = F.conv3d(xb[n:n + 1, :, lo:hi], wq, padding=1)[0, :, z - lo].permute(1, 2, 0)
            dd = (y[n, z].double().cpu() - ref).abs()
            assert bool((dd <= ref.abs() * 2.0 ** -8 + 1e-6 * ref.abs().max()).all()), (n, z, dd.max().item())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,c,dims", [(2, 64, (6, 7, 9)), (3, 256, (5, 4, 3)), (1, 32, (9, 11, 13)), (2, 128, (24, 24, 24))])
def test_gn_apply_materialised(gpu, dt, n, c, dims):
    """relu(gn(x)) materialised (u3d_gn_apply, sample-per-grid-row kernel) against the prologue formula."""
    from u3d import ops
    torch.manual_seed(9)
    x = (torch.randn((n,) + dims + (c,), device=gpu) * 1.5 + 0.3).to(dt)
    st = ops.gn_stats(x, 16)
    ga = 1 + 0.1 * torch.randn(c, device=gpu)
    be = 0.1 * torch.randn(c, device=gpu)
    y = ops.gn_apply(x, st, ga, be, 16)
    if dt == torch.float32:
        xf = x.cpu()
        g = torch.arange(c) // (c // 16)
        s = st.cpu()
        sc = s[:, g, 1] * ga.cpu()[None]
        sh = be.cpu()[None] - s[:, g, 0] * sc
        ref = torch.clamp_min(xf * sc.view(n, 1, 1, 1, c) + sh.view(n, 1, 1, 1, c), 0).double()
        assert (y.double().cpu() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    else:
        ref = _act_ref(x, st, ga, be, 16)
        assert (y.double().cpu() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


def test_bf16_stem_bench_size(gpu):
    """conv1 (1 -> 32, 2 x 96^3) as the bench runs it: sampled output planes (first, middle, last of each sample)
    against fp64 on the bf16-rounded input, 1e-2 of the plane's max |y| (the kernel keeps the fp32 input, so the
    bf16-rounded reference bounds its error from above)."""
    from u3d import ops
    torch.manual_seed(5)
    x = torch.rand((2, 1, 96, 96, 96), device=gpu) * 2 - 1
    w = torch.randn(32, 1, 3, 3, 3, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    y = ops.stem_fwd(x, pf, 32, 1, torch.bfloat16)
    wq = pf.float().cpu()[:, :32, :1].permute(1, 2, 0).reshape(32, 1, 3, 3, 3).double()
    xb = x.to(torch.bfloat16).double().cpu()
    for n in range(2):
        for z in (0, 47, 95):
            lo, hi = max(0, z - 1), min(96, z + 2)
            ref = F.conv3d(xb[n:n + 1, :, lo:hi], wq, padding=1)[0, :, z - lo].permute(1, 2, 0)
            err = (y[n, z].double().cpu() - ref).abs().max().item()
            assert err < 1e-2 * ref.abs().max().item(), (n, z, err)


@pytest.mark.parametrize("cin,cout,dims", [(32, 16, (48, 48, 48)), (64, 8, (5, 7, 9)), (16, 32, (3, 11, 13))])
def test_head_transposed_bitwise_equal(gpu, cin, cout, dims):
    """The transposed-MFMA head (16-B stores; default for cout % 8 == 0) against the untransposed form
    (option HEAD_TR=0): the same products summed in the same order, the same bf16 rounding -> bitwise equal."""
    from u3d import ops
    n = 2
    x, _, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 9)
    w = torch.randn(cout, cin, 1, 1, 1, device=gpu)
    pf, pd, _ = ops.wstd_fwd(w, torch.bfloat16, False)
    b = torch.randn(cout, device=gpu)
    dy = torch.randn(x.shape[:-1] + (cout,), device=gpu)
    out = []
    for tr in (1, 0):
        with ops.option("HEAD_TR", tr):
            y = ops.head_fwd(x, pf, cout, b, (st, ga, be, G))
            dA, dyb = ops.head_bwd(dy, pd, cin)
            torch.cuda.synchronize()
        out.append((y, dA, dyb))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1].view(torch.int16), out[1][1].view(torch.int16))
    assert torch.equal(out[0][2].view(torch.int16), out[1][2].view(torch.int16))


@pytest.mark.parametrize("n,c,dims,skip", [(2, 32, (48, 48, 48), True), (1, 64, (5, 1, 7), True), (2, 16, (3, 4, 1), False),
                                          (1, 128, (12, 12, 12), True), (1, 8, (1, 1, 1), True)])
def test_upsample_quad_bitwise_equals_one_output(gpu, n, c, dims, skip):
    """bf16 trilinear x2 upsample (+ skip): the 2 x 2-outputs-per-thread kernel (UP_QUAD=1, round 4) is bitwise equal
    to the one-output kernel (same Lerp weights, same expression; boundary taps selected, not clamped differently)."""
    from u3d import ops
    torch.manual_seed(13)
    x = torch.randn((n,) + dims + (c,), device=gpu).to(torch.bfloat16)
    s = torch.randn((n,) + tuple(2 * v for v in dims) + (c,), device=gpu).to(torch.bfloat16) if skip else None
    with ops.option("UP_QUAD", 0):
        a = ops.upsample2x_add(x, s)
    with ops.option("UP_QUAD", 1):
        b = ops.upsample2x_add(x, s)
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
