"""bf16 stride-2 3^3 forward conv (csrc/conv_s2.hip, u3d_conv_fwd_s2) against an fp64 CPU reference on the same
bf16-rounded operands and bf16-rounded GN+ReLU prologue (as test_gpu_bf16.py: 1e-2 of max |y|) and against the implicit
GEMM it replaces. Shapes: ragged bricks in every dim (output not a multiple of 2 x 4 x 16), odd input extents, cin not a
multiple of 32 (zero-filled last chunk planes), cout not a multiple of 32, several samples, more units than workgroups
(the persistent walk), with and without the GN prologue. Reference: F.conv3d(stride=2, padding=1) in Conv3d.forward
(unet3D.py:27), conv1 of the first NoBottleneck of layer1..4 (_make_layer :1666-1686)."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_bf16 import _act_ref

pytestmark = pytest.mark.gpu

SHAPES = [(2, 32, 64, (12, 16, 34)), (1, 32, 64, (9, 13, 31)), (2, 64, 128, (16, 16, 48)), (3, 40, 48, (7, 10, 40)),
          (1, 128, 256, (24, 24, 24)), (2, 256, 256, (12, 12, 32)), (1, 32, 32, (5, 3, 70)), (2, 64, 96, (4, 20, 24))]


@pytest.fixture
def s2_on():
    from u3d import ops
    saved = (ops.USE_S2_FWD, ops.S2_FWD_MIN_W)
    ops.USE_S2_FWD, ops.S2_FWD_MIN_W = True, 1
    yield ops
    ops.USE_S2_FWD, ops.S2_FWD_MIN_W = saved


@pytest.mark.parametrize("n,cin,cout,dims", SHAPES)
@pytest.mark.parametrize("gn", [True, False])
def test_conv_fwd_s2(gpu, s2_on, n, cin, cout, dims, gn):
    ops = s2_on
    torch.manual_seed(cin * 7 + cout)
    x = (torch.randn((n,) + dims + (cin,), device=gpu) * 1.4 + 0.2).to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, 3, device=gpu)
    G = 16 if cin % 16 == 0 else 8
    st = ops.gn_stats(x, G) if gn else None
    ga = 1 + 0.1 * torch.randn(cin, device=gpu)
    be = 0.1 * torch.randn(cin, device=gpu)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    g = (st, ga, be, G) if gn else None
    y = ops.conv_fwd(x, pf, cout, 3, 2, g)
    a = _act_ref(x, st, ga, be, G).permute(0, 4, 1, 2, 3)
    wq = pf.float().cpu()[:, :cout, :cin].permute(1, 2, 0).reshape(cout, cin, 3, 3, 3).double()
    ref = F.conv3d(a, wq, stride=2, padding=1).permute(0, 2, 3, 4, 1)
    assert y.shape == ref.shape
    scale = ref.abs().max().item()
    err = (y.double().cpu() - ref).abs().max().item()
    assert err < 1e-2 * scale, err
    ops.USE_S2_FWD = False
    try:
        y0 = ops.conv_fwd(x, pf, cout, 3, 2, g)
    finally:
        ops.USE_S2_FWD = True  # restored to the caller's value by the fixture
    assert (y.double() - y0.double()).abs().max().item() < 1e-2 * scale
