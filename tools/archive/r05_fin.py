"""Round 5: the in-launch finalize (last-arriving workgroup, ops.FUSED_FINALIZE) against the separate finalize
launch, per site, at the bench sizes (graph-replayed, per call incl. the launch gap), and the batched slab sum alone.
Usage: python tools/r05_fin.py"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402
from kbench import t_, conv_case, dev, bf  # noqa: E402
from u3d import ops  # noqa: E402


def both(label, fn):
    r = []
    for ff in (False, True):
        ops.FUSED_FINALIZE = ff
        r.append(t_(fn))
    ops.FUSED_FINALIZE = True
    print(f"{label:34s} separate {r[0]:7.1f} us   in-launch {r[1]:7.1f} us   diff {r[1] - r[0]:+6.1f}", flush=True)


for s, c, res in [(96, 32, True), (96, 32, False), (48, 64, True), (48, 64, False), (24, 128, True)]:
    x, pf, pd, g, r, dy, _ = conv_case(2, c, c, s, 3, 1, True, res)
    both(f"fwd+stats {s}^3 c{c} res={res}", lambda: ops.conv_fwd_stats(x, pf, c, 3, 1, g, r))

for s, c in [(96, 32)]:
    x, pf, pd, g, r, dy, _ = conv_case(2, c, c, s, 3, 1, True)
    dg, db = torch.zeros(c, device=dev), torch.zeros(c, device=dev)

    def gnb():
        rr = ops.conv_dgrad_gn(dy, pd, c, x, 3, 1, g, dgb=lambda: (dg, db))
        if isinstance(rr[1], tuple):
            return ops.gn_bwd_apply_coef(rr[0], x, rr[1][1], g[3])
        return ops.gn_bwd_parts(rr[0], x, rr[1], g[0], g[1], g[2], g[3], dgamma=dg, dbeta=db)
    both(f"dgrad+GN-bwd {s}^3 c{c}", gnb)

for s, c in [(96, 32), (48, 64), (24, 128), (12, 256)]:
    x, pf, pd, g, r, dy, _ = conv_case(2, c, c, s, 3, 1, True)
    w = torch.randn(c, c, 3, 3, 3, device=dev) * 0.05
    _, _, st = ops.wstd_fwd(w, bf, True, need_dgrad=False)
    part, ns = ops.conv_wgrad(dy, x, 3, 1, g)
    dw = torch.empty_like(w)
    t_sum = t_(lambda: ops.wstd_bwd_batch([(part, ns, w, st, True, dw, False)]))
    p1 = part[:1].clone()
    t_one = t_(lambda: ops.wstd_bwd_batch([(p1, 1, w, st, True, dw, False)]))
    mb = part.numel() * 4 / 1e6
    print(f"slab sum {s}^3 c{c}: {ns} slabs {mb:6.1f} MB  sum+wstd {t_sum:6.1f} us  wstd alone {t_one:6.1f} us  "
          f"sum ~{(t_sum - t_one):6.1f} us = {mb * 1e-3 / max(t_sum - t_one, 1e-3) * 1e3:5.2f} TB/s", flush=True)
