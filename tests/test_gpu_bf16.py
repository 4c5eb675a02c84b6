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
          (1, 64, 32, (10, 6, 8), 1), (2, 128, 128, (4, 4, 4), 1), (1, 24, 24, (7, 9, 11), 1)]


@pytest.fixture(params=["auto", "gen_brick", "igemm"])
def conv_path(request):
    """auto = production routing; gen_brick = force the generic halo-brick kernel; igemm = force implicit GEMM."""
    from u3d import ops
    saved = (ops.BRICK_MIN_WG, ops.USE_CONV32_BRICK, ops.USE_GEN_BRICK)
    if request.param == "gen_brick":
        ops.BRICK_MIN_WG, ops.USE_CONV32_BRICK = 0, False
    elif request.param == "igemm":
        ops.USE_CONV32_BRICK, ops.USE_GEN_BRICK = False, False
    yield request.param
    ops.BRICK_MIN_WG, ops.USE_CONV32_BRICK, ops.USE_GEN_BRICK = saved


@pytest.mark.parametrize("n,cin,cout,dims,s", SHAPES)
def test_bf16_conv_fwd(gpu, conv_path, n, cin, cout, dims, s):
    from u3d import ops
    x, w, st, ga, be, G = _case(gpu, n, cin, cout, dims, True, 1)
    pf, pd, wst = ops.wstd_fwd(w, torch.bfloat16, True)
    y = ops.conv_fwd(x, pf, cout, 3, s, (st, ga, be, G))
    a = _act_ref(x, st, ga, be, G).permute(0, 4, 1, 2, 3)
    wq = pf.float().cpu()[:, :cout, :cin].permute(1, 2, 0).reshape(cout, cin, 3, 3, 3).double()
    ref = F.conv3d(a, wq, stride=s, padding=1).permute(0, 2, 3, 4, 1)
    err = (y.double().cpu() - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("n,cin,cout,dims,s", SHAPES)
def test_bf16_conv_dgrad(gpu, conv_path, n, cin, cout, dims, s):
    from u3d import ops
    if s == 2 and any(d % 2 for d in dims):
        pytest.skip("stride-2 dgrad needs even dims (as the trunk has)")
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


@pytest.mark.parametrize("brick", [True, False])
@pytest.mark.parametrize("n,cin,cout,dims,s", SHAPES)
def test_bf16_conv_wgrad(gpu, n, cin, cout, dims, s, brick):
    from u3d import ops
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
