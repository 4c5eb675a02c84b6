"""Fixed cost of a ring launch: the 32-channel ring forward (GN prologue + statistics) and data gradient on volumes of
1..4 output planes per workgroup (graph-replayed, per call), against the 2 x 96^3 launch. Usage: python tools/r05_tiny.py"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402
from kbench import t_, dev, bf  # noqa: E402
from u3d import ops  # noqa: E402

for (n, d, h, w) in [(1, 1, 8, 32), (2, 8, 32, 32), (2, 16, 96, 96), (2, 96, 96, 96)]:
    x = torch.randn((n, d, h, w, 32), device=dev).to(bf)
    wt = torch.randn(32, 32, 3, 3, 3, device=dev) * 0.05
    pf, pd, _ = ops.wstd_fwd(wt, bf, True)
    g = (ops.gn_stats(x, 16), torch.ones(32, device=dev), torch.zeros(32, device=dev), 16)
    us_f = t_(lambda: ops.conv_fwd_stats(x, pf, 32, 3, 1, g))
    us_d = t_(lambda: ops.conv_dgrad(x, pd, 32, x.shape[:4], 3, 1))
    print(f"{n}x{d}x{h}x{w}: fwd+stats {us_f:7.1f} us   dgrad {us_d:7.1f} us", flush=True)
