"""The weight gradient's slab sum right after its launch (round 5, u3d_wgrad_sum_slabs / ops.sum_slabs, option
U3D_EAGER_SLAB_SUM) against the sum inside the batched standardisation backward (u3d_wstd_bwd_batch): the same kernel,
slab groups and order, so the standardised weight gradient is BITWISE equal. Cases: the bench levels' weight-gradient
kernels (96^3 DMA ring, 48^3 ring, 24^3 / 12^3 register rings, a 1^3 conv). Reference: autograd of the weight-
standardised Conv3d (unet3D.py:16-27)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,cin,cout,dims,k", [(2, 32, 32, (96, 96, 96), 3), (2, 64, 64, (48, 48, 48), 3),
                                               (2, 128, 128, (24, 24, 24), 3), (2, 256, 256, (12, 12, 12), 3),
                                               (2, 64, 128, (24, 24, 24), 1)], ids=str)
def test_eager_slab_sum_bitwise(gpu, n, cin, cout, dims, k):
    from u3d import ops
    torch.manual_seed(3)
    x = (torch.randn((n,) + dims + (cin,), device=gpu)).to(torch.bfloat16)
    dy = (torch.randn((n,) + dims + (cout,), device=gpu) * 0.5).to(torch.bfloat16)
    w = torch.randn(cout, cin, k, k, k, device=gpu) * 0.05
    _, _, st = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    part, ns = ops.conv_wgrad(dy, x, k, 1)
    part2 = part.clone()
    dw_a, dw_b = torch.empty_like(w), torch.empty_like(w)
    ops.wstd_bwd_batch([(part, ns, w, st, True, dw_a, False)])
    p2, ns2 = ops.sum_slabs(part2, ns, cout, cin)
    assert ns2 == 1
    ops.wstd_bwd_batch([(p2, 1, w, st, True, dw_b, False)])
    torch.cuda.synchronize()
    assert torch.equal(dw_a, dw_b)
    assert torch.equal(part[0], p2[0])  # the batched form sums into slab 0 as well
