"""Kernel micro-benchmarks on cuda:0 (HIP events, per-launch average). Usage: python tools/kbench.py [case ...]
Cases reproduce the trunk's launches at 2 x 96^3 (bf16) so rocprofv3 PMC passes can target one kernel."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
import torch  # noqa: E402
from u3d import ops  # noqa: E402

dev = torch.device("cuda:0")
for kv in os.environ.get("KB_SET", "").split(","):  # e.g. KB_SET=USE_SMALL_CONV=0,SMALL_MAX_VOX=1e9
    if kv:
        k, v = kv.split("=")
        cur = getattr(ops, k)
        setattr(ops, k, v if isinstance(cur, str) else type(cur)(float(v)))
bf = torch.bfloat16


def t_(fn, reps=20):
    """GPU time per call: `reps` calls captured in one hipGraph and replayed (no host launch overhead)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * reps) * 1e3


def conv_case(n, cin, cout, s, k, stride, gn=True, res=False):
    x = torch.randn((n, s, s, s, cin), device=dev).to(bf)
    w = torch.randn(cout, cin, k, k, k, device=dev)
    pf, pd, _ = ops.wstd_fwd(w, bf, True)
    G = 16
    g = (ops.gn_stats(x, G), torch.ones(cin, device=dev), torch.zeros(cin, device=dev), G) if gn else None
    os_ = ops.out_dim(s, k, stride)
    r = torch.randn((n, os_, os_, os_, cout), device=dev).to(bf) if res else None
    dy = torch.randn((n, os_, os_, os_, cout), device=dev).to(bf)
    flop = 2.0 * n * os_ ** 3 * k ** 3 * cin * cout
    return x, pf, pd, g, r, dy, flop


CASES = {}


def case(name):
    def deco(f):
        CASES[name] = f
        return f
    return deco


def _fwd(n, cin, cout, s, k, stride, gn=True, res=False):
    x, pf, pd, g, r, dy, flop = conv_case(n, cin, cout, s, k, stride, gn, res)
    if g is not None and cout == 32:  # production path: GroupNorm statistics from the ring epilogue
        us = t_(lambda: ops.conv_fwd_stats(x, pf, cout, k, stride, g, r))
    else:
        us = t_(lambda: ops.conv_fwd(x, pf, cout, k, stride, g, r))
    return us, flop


def _dgrad(n, cin, cout, s, k, stride):
    x, pf, pd, g, r, dy, flop = conv_case(n, cin, cout, s, k, stride, False)
    us = t_(lambda: ops.conv_dgrad(dy, pd, cin, x.shape[:4], k, stride))
    return us, flop


def _dgrad_gn(n, c, s):
    """the production 96^3 data gradient: ring with the GroupNorm-backward partials fused in its epilogue"""
    x, pf, pd, g, r, dy, flop = conv_case(n, c, c, s, 3, 1, True)
    us = t_(lambda: ops.conv_dgrad_gn(dy, pd, c, x, 3, 1, g))
    return us, flop


def _wgrad(n, cin, cout, s, k, stride):
    x, pf, pd, g, r, dy, flop = conv_case(n, cin, cout, s, k, stride, True)
    us = t_(lambda: ops.conv_wgrad(dy, x, k, stride, g, brick={"ring": "ring", "brick": True}.get(os.environ.get("KB_WGRAD", ""))))
    return us, flop


for (lvl, s, c) in [("96", 96, 32), ("48", 48, 64), ("24", 24, 128), ("12", 12, 256), ("6", 6, 256)]:
    CASES[f"fwd{lvl}"] = (lambda s=s, c=c: _fwd(2, c, c, s, 3, 1, True, True))
    CASES[f"dgrad{lvl}"] = (lambda s=s, c=c: _dgrad(2, c, c, s, 3, 1))
    CASES[f"wgrad{lvl}"] = (lambda s=s, c=c: _wgrad(2, c, c, s, 3, 1))
CASES["dgrad96gn"] = lambda: _dgrad_gn(2, 32, 96)
for (_lvl, _s, _c) in [("96", 96, 32), ("48", 48, 64), ("24", 24, 128), ("12", 12, 256)]:
    CASES[f"wgsum{_lvl}"] = (lambda s=_s, c=_c: _wgrad_sum(2, c, s))  # weight gradient + its slab sum


def _wgrad_sum(n, c, s):
    """the stride-1 ring weight gradient and the sum of its split slabs (what the step pays per weight, before the
    standardisation backward)"""
    x, pf, pd, g, r, dy, flop = conv_case(n, c, c, s, 3, 1, True)

    def f():
        part, ns = ops.conv_wgrad(dy, x, 3, 1, g)
        ops.sum_slabs(part, ns, c, c)
    return t_(f), flop
CASES["fwd96nr"] = lambda: _fwd(2, 32, 32, 96, 3, 1, True, False)   # GN prologue + statistics, no residual
CASES["wgrad96nogn"] = lambda: _wgrad_plain(2, 32, 96)               # the weight-gradient ring without its GN prologue


def _wgrad_plain(n, c, s):
    x, pf, pd, g, r, dy, flop = conv_case(n, c, c, s, 3, 1, False)
    us = t_(lambda: ops.conv_wgrad(dy, x, 3, 1, None))
    return us, flop
CASES["dgrad48gn"] = lambda: _dgrad_gn(2, 64, 48)   # persistent brick + GN-backward partials (round 4)


def _fwd_stats(n, c, s, res):
    """the production brick forward: GN prologue (+ residual) + GroupNorm(16) statistics of the output from its epilogue"""
    x, pf, pd, g, r, dy, flop = conv_case(n, c, c, s, 3, 1, True, res)
    return t_(lambda: ops.conv_fwd_stats(x, pf, c, 3, 1, g, r)), flop


def _up(n, c, s):
    """trilinear x2 upsample + skip add (decoder, unet3D.py:1646) into an s^3 output: (us, bytes moved)"""
    x = torch.randn((n, s // 2, s // 2, s // 2, c), device=dev).to(bf)
    sk = torch.randn((n, s, s, s, c), device=dev).to(bf)
    return t_(lambda: ops.upsample2x_add(x, sk)), 2.0 * (x.numel() + 2 * sk.numel())


def _upb(n, c, s):
    """trilinear x2 upsample backward (adjoint gather) from an s^3 gradient"""
    dy = torch.randn((n, s, s, s, c), device=dev).to(bf)
    shape = (n, s // 2, s // 2, s // 2, c)
    return t_(lambda: ops.upsample2x_bwd(dy, shape)), 2.0 * (dy.numel() + dy.numel() // 8)


def _up_stats(n, c, s):
    """the decoder's upsample + skip with the output's GroupNorm(16) statistics from its epilogue (the step's form)"""
    x = torch.randn((n, s // 2, s // 2, s // 2, c), device=dev).to(bf)
    sk = torch.randn((n, s, s, s, c), device=dev).to(bf)
    return t_(lambda: ops.upsample2x_add_stats(x, sk)), 2.0 * (x.numel() + 2 * sk.numel())


CASES["up96st"] = lambda: _up_stats(2, 32, 96)
CASES["up48st"] = lambda: _up_stats(2, 64, 48)
CASES["up96"] = lambda: _up(2, 32, 96)
CASES["upb96"] = lambda: _upb(2, 32, 96)
CASES["upb48"] = lambda: _upb(2, 64, 48)
CASES["up48"] = lambda: _up(2, 64, 48)
CASES["fwd48st"] = lambda: _fwd_stats(2, 64, 48, True)
CASES["fwd48st_nores"] = lambda: _fwd_stats(2, 64, 48, False)
CASES["fwd24st"] = lambda: _fwd_stats(2, 128, 24, True)
CASES["dgrad24gn"] = lambda: _dgrad_gn(2, 128, 24)


def _gnb(n, c, s, fused):
    """data gradient + the whole GroupNorm backward (dx, dgamma, dbeta): fused partials + parts finalize + apply, or
    the separate data gradient + partial pass + apply"""
    x, pf, pd, g, r, dy, flop = conv_case(n, c, c, s, 3, 1, True)
    dg, db = torch.zeros(c, device=dev), torch.zeros(c, device=dev)

    def f():
        if fused:
            da, parts = ops.conv_dgrad_gn(dy, pd, c, x, 3, 1, g)
            ops.gn_bwd_parts(da, x, parts, g[0], g[1], g[2], g[3], dgamma=dg, dbeta=db)
        else:
            da = ops.conv_dgrad(dy, pd, c, x.shape[:4], 3, 1)
            ops.gn_bwd(da, x, g[0], g[1], g[2], g[3], dgamma=dg, dbeta=db)
    return t_(f), flop


for (lvl, s, c) in [("96", 96, 32), ("48", 48, 64), ("24", 24, 128)]:
    CASES[f"gnb{lvl}f"] = (lambda s=s, c=c: _gnb(2, c, s, True))
    CASES[f"gnb{lvl}s"] = (lambda s=s, c=c: _gnb(2, c, s, False))
CASES["fwd12nogn"] = lambda: _fwd(2, 256, 256, 12, 3, 1, False, False)
CASES["wgrad_s2_96"] = lambda: _wgrad(2, 32, 64, 96, 3, 2)
CASES["wgrad_s2_48"] = lambda: _wgrad(2, 64, 128, 48, 3, 2)
CASES["wgrad_s2_24"] = lambda: _wgrad(2, 128, 256, 24, 3, 2)
CASES["fwd_s2_24"] = lambda: _fwd(2, 128, 256, 24, 3, 2, True, False)
CASES["fwd_s2_24nogn"] = lambda: _fwd(2, 128, 256, 24, 3, 2, False, False)
CASES["fwd_s2_48"] = lambda: _fwd(2, 64, 128, 48, 3, 2, True, False)
CASES["fwd_s2_48nogn"] = lambda: _fwd(2, 64, 128, 48, 3, 2, False, False)
CASES["fwd_s2_12"] = lambda: _fwd(2, 256, 256, 12, 3, 2, True, False)
CASES["fwd_s2_12nogn"] = lambda: _fwd(2, 256, 256, 12, 3, 2, False, False)
CASES["wgrad_s2_48nogn"] = lambda: _wgrad_nogn(2, 64, 128, 48, 2)
CASES["wgrad_s2_24nogn"] = lambda: _wgrad_nogn(2, 128, 256, 24, 2)
CASES["wgrad_s2_96nogn"] = lambda: _wgrad_nogn(2, 32, 64, 96, 2)
CASES["gn_apply48"] = lambda: _gn_apply(2, 64, 48)
CASES["gn_apply24"] = lambda: _gn_apply(2, 128, 24)


def _wgrad_nogn(n, cin, cout, s, stride):
    x, pf, pd, g, r, dy, flop = conv_case(n, cin, cout, s, 3, stride, False)
    us = t_(lambda: ops.conv_wgrad(dy, x, 3, stride, None))
    return us, flop


def _gn_apply(n, c, s):
    """relu(gn(x)) materialised (bf16 NDHWC): the cost of normalising a stride-2 conv's input once"""
    x = torch.randn((n, s, s, s, c), device=dev).to(bf)
    st = ops.gn_stats(x, 16)
    ga, be = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    us = t_(lambda: ops.gn_apply(x, st, ga, be, 16))
    return us, 0.0
CASES["dgrad_s2_24"] = lambda: _dgrad(2, 128, 256, 24, 3, 2)
CASES["dgrad_s2_96"] = lambda: _dgrad(2, 32, 64, 96, 3, 2)
CASES["dgrad_s2_48"] = lambda: _dgrad(2, 64, 128, 48, 3, 2)
CASES["dgrad_s2_12"] = lambda: _dgrad(2, 256, 256, 12, 3, 2)
CASES["fwd6nogn"] = lambda: _fwd(2, 256, 256, 6, 3, 1, False, False)
CASES["dgrad1_s2_96"] = lambda: _dgrad(2, 32, 64, 96, 1, 2)
CASES["dgrad1_s2_48"] = lambda: _dgrad(2, 64, 128, 48, 1, 2)
CASES["fwd1_s2_96"] = lambda: _fwd(2, 32, 64, 96, 1, 2, True, False)
CASES["fwd96_nores"] = lambda: _fwd(2, 32, 32, 96, 3, 1, True, False)


def _fwd_s2_ring(n=2, s=96):
    """the production stride-2 forward (layer1.0.conv1, 32 -> 64 with GN prologue + output stats: conv_s2.hip)"""
    x, pf, pd, g, r, dy, flop = conv_case(n, 32, 64, s, 3, 2, True)
    return t_(lambda: ops.conv_fwd_stats(x, pf, 64, 3, 2, g)), flop


CASES["fwds2ring"] = _fwd_s2_ring
CASES["wgrad1_96"] = lambda: _wgrad(2, 32, 16, 96, 1, 1)      # the head's 1^3 weight gradient
CASES["wgrad1_s2_96"] = lambda: _wgrad(2, 32, 64, 96, 1, 2)   # layer1 downsample
CASES["fwd96_nogn"] = lambda: _fwd(2, 32, 32, 96, 3, 1, False, True)
CASES["fwd96_plain"] = lambda: _fwd(2, 32, 32, 96, 3, 1, False, False)
CASES["head96"] = lambda: _fwd(2, 32, 16, 96, 1, 1, True, False)


def _hlb(n, s, mode):
    """the head's fused loss + data-gradient backward at 2 x 96^3 (cin 32, 16 classes): "plain" alone, "gn" with the
    prologue GN's backward partials, "sep" / "fused" plus the whole GroupNorm backward (separate partial pass or parts)"""
    shp = (n, s, s, s)
    lg = torch.randn(shp + (16,), device=dev) * 3
    lab = torch.randint(0, 16, shp, device=dev).float()
    wt = torch.ones(16, device=dev)
    _, sums = ops.partial_loss_fwd(lg, lab, wt, True, True)
    go = torch.ones(1, device=dev)
    _, pd, _ = ops.wstd_fwd(torch.randn(16, 32, 1, 1, 1, device=dev), bf, False)
    x0 = torch.randn(shp + (32,), device=dev).to(bf)
    g = (ops.gn_stats(x0, 8), torch.ones(32, device=dev), torch.zeros(32, device=dev), 8)
    dg, db, dbb = torch.zeros(32, device=dev), torch.zeros(32, device=dev), torch.zeros(16, device=dev)

    def f():
        if mode in ("gn", "fused"):
            da, _, parts = ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, dbias=dbb, x0=x0, gn=g)
            if mode == "fused":
                ops.gn_bwd_parts(da, x0, parts, g[0], g[1], g[2], 8, dgamma=dg, dbeta=db)
        else:
            da, _ = ops.head_loss_bwd(lg, lab, wt, sums, go, pd, 32, dbias=dbb)
            if mode == "sep":
                ops.gn_bwd(da, x0, g[0], g[1], g[2], 8, dgamma=dg, dbeta=db)
    return t_(f), 0.0


for _m in ("plain", "gn", "sep", "fused"):
    CASES[f"hlb96{_m}"] = (lambda m=_m: _hlb(2, 96, m))


def _slabsum(ns, co, ci):
    """the slab sum of one weight gradient [ns, 27, co, ci] fp32 (u3d_wgrad_sum_slabs): the batched end-of-step sum's
    per-weight work (96^3: 256 slabs of 27 x 32 x 32; 48^3: 64 of 27 x 64 x 64; 24^3: 16 of 128^2; 12^3: 4 of 256^2)"""
    part = torch.randn(ns, 27, co, ci, device=dev)
    us = t_(lambda: ops.sum_slabs(part, ns, co, ci))
    print(f"   ({part.numel() * 4 / us / 1e6:.2f} TB/s read)")
    return us, 0.0


for (_lvl, _ns, _c) in (("96", 256, 32), ("48", 64, 64), ("24", 16, 128), ("12", 4, 256)):
    CASES[f"slabsum{_lvl}"] = (lambda ns=_ns, c=_c: _slabsum(ns, c, c))


def _queue(fn):
    def run():
        saved = ops.RING_QUEUE
        ops.RING_QUEUE = True
        try:
            return fn()
        finally:
            ops.RING_QUEUE = saved
    return run


CASES["fwd96q"] = _queue(CASES["fwd96"])
CASES["dgrad96q"] = _queue(CASES["dgrad96"])

def _stem_plain(n=2, s=96):
    x = torch.rand((n, 1, s, s, s), device=dev)
    w = torch.randn(32, 1, 3, 3, 3, device=dev)
    pf, _, _ = ops.wstd_fwd(w, bf, True, need_dgrad=False)
    return t_(lambda: ops.stem_fwd(x, pf, 32, 1, bf)), 2.0 * n * s ** 3 * 27 * 32


def _stem_stats(n=2, s=96):
    """the bench's conv1: 1 -> 32 with the output GroupNorm(16) statistics from the epilogue (stem1_mfma_kernel<true>)"""
    x = torch.rand((n, 1, s, s, s), device=dev)
    w = torch.randn(32, 1, 3, 3, 3, device=dev)
    pf, _, _ = ops.wstd_fwd(w, bf, True, need_dgrad=False)
    return t_(lambda: ops.stem_fwd_stats(x, pf, 32, 1, bf)), 2.0 * n * s ** 3 * 27 * 32


CASES_EXTRA = {"fwd_s2_96": lambda: _fwd(2, 32, 64, 96, 3, 2, True, False),
               "fwd_s2_48": lambda: _fwd(2, 64, 128, 48, 3, 2, True, False),
               "fwd_s2_12": lambda: _fwd(2, 256, 256, 12, 3, 2, True, False),
               "fwd48_plain": lambda: _fwd(2, 64, 64, 48, 3, 1, False, False),
               "fwd48_gn": lambda: _fwd(2, 64, 64, 48, 3, 1, True, False),
               "fwd48_res": lambda: _fwd(2, 64, 64, 48, 3, 1, False, True),
               "fwd24_plain": lambda: _fwd(2, 128, 128, 24, 3, 1, False, False),
               "stem96": lambda: _stem_plain(),
               "stem96st": lambda: _stem_stats()}
CASES.update(CASES_EXTRA)


for (nm, cx, cy, s_, st_) in [("c1_s2_96", 32, 64, 96, 2), ("c1_s2_48", 64, 128, 48, 2), ("c1_s2_24", 128, 256, 24, 2),
                             ("c1_s2_12", 256, 256, 12, 2), ("c1_48", 64, 32, 48, 1), ("c1_24", 128, 64, 24, 1),
                             ("c1_12", 256, 128, 12, 1), ("c1_6", 256, 256, 6, 1)]:
    CASES[nm] = (lambda cx=cx, cy=cy, s_=s_, st_=st_: _fwd(2, cx, cy, s_, 1, st_, True, False))
    if st_ == 1:
        CASES["d" + nm] = (lambda cx=cx, cy=cy, s_=s_: _dgrad(2, cx, cy, s_, 1, 1))


def _upp(bwd, n=2, s=48, c=32):
    x = torch.randn((n, s, s, s, c), device=dev).to(bf)
    sk = torch.randn((n, 2 * s, 2 * s, 2 * s, c), device=dev).to(bf)
    fn = (lambda: ops.upsample2x_bwd(sk, tuple(x.shape))) if bwd else (lambda: ops.upsample2x_add(x, sk))
    return t_(fn), 0.0


CASES["upf96"] = lambda: _upp(False)
CASES["upf48"] = lambda: _upp(False, 2, 24, 64)
CASES["upb96"] = lambda: _upp(True)
CASES["upb48"] = lambda: _upp(True, 2, 24, 64)
CASES["upb24"] = lambda: _upp(True, 2, 12, 128)
CASES["upb12"] = lambda: _upp(True, 2, 6, 256)
CASES["dec24_c1"] = lambda: _fwd(2, 128, 64, 24, 3, 1, True, False)
CASES["dec24_c2"] = lambda: _fwd(2, 64, 64, 24, 3, 1, True, True)
CASES["ddec24_c1"] = lambda: _dgrad(2, 128, 64, 24, 3, 1)
CASES["ddec24_c2"] = lambda: _dgrad(2, 64, 64, 24, 3, 1)
CASES["dec48_c1"] = lambda: _fwd(2, 64, 32, 48, 3, 1, True, False)
CASES["ddec48_c1"] = lambda: _dgrad(2, 64, 32, 48, 3, 1)
CASES["dec12_c1"] = lambda: _fwd(2, 256, 128, 12, 3, 1, True, False)
CASES["dec12_c2"] = lambda: _fwd(2, 128, 128, 12, 3, 1, True, True)


def _gn(kind, s, c, n=2, G=16):
    x = torch.randn((n, s, s, s, c), device=dev).to(bf)
    da = torch.randn_like(x)
    da2 = torch.randn_like(x)
    h2 = ops.out_dim(s, 1, 2)
    da2c = torch.randn((n, h2, h2, h2, c), device=dev).to(bf)
    ga, be = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1
    st = ops.gn_stats(x, G)
    dx = torch.empty_like(x)
    fns = {"stats": lambda: ops.gn_stats(x, G),
           "apply": lambda: ops.gn_apply(x, st, ga, be, G),
           "bwd": lambda: ops.gn_bwd(da, x, st, ga, be, G, dx=dx, accumulate=True),
           "bwd2": lambda: ops.gn_bwd2(da, da2, x, st, (ga, be), (ga, be), G, dx=dx, accumulate=True),
           "bwd2s": lambda: ops.gn_bwd2(da, da2c, x, st, (ga, be), (ga, be), G, dx=dx, accumulate=True, da2_s2=True)}
    return t_(fns[kind]), 0.0


for (lvl, s, c) in [("96", 96, 32), ("48", 48, 64), ("24", 24, 128), ("12", 12, 256), ("6", 6, 256)]:
    for kind in ("stats", "apply", "bwd", "bwd2", "bwd2s"):
        CASES[f"gn{kind}{lvl}"] = (lambda kind=kind, s=s, c=c: _gn(kind, s, c))


def _loss(n, s, C, bwd):
    """EDiceLoss_partial forward (per-class sums over the fp32 logits) / backward (dlogits), 2 x 96^3 x 16"""
    lg = torch.randn((n, s, s, s, C), device=dev)
    lab = torch.randint(0, C, (n, s, s, s), device=dev).float()
    wt = torch.ones(C, device=dev)
    if not bwd:
        return t_(lambda: ops.partial_loss_fwd(lg, lab, wt)), 0.0
    _, sums = ops.partial_loss_fwd(lg, lab, wt)
    go = torch.ones(1, device=dev)
    return t_(lambda: ops.partial_loss_bwd(lg, lab, wt, sums, go)), 0.0


def _stemw(n=2, s=96):
    x = torch.randn((n, 1, s, s, s), device=dev)
    dy = torch.randn((n, s, s, s, 32), device=dev).to(bf)
    return t_(lambda: ops.stem_wgrad(dy, x, 1)), 2.0 * n * s ** 3 * 27 * 32


def _head(bwd, n=2, s=96, cin=32, cout=16):
    """precls head (head.hip): GN+ReLU+1^3 conv to fp32 logits (+ bias) / its data gradient from fp32 dlogits"""
    x, pf, pd, g, r, dy, flop = conv_case(n, cin, cout, s, 1, 1, True)
    b = torch.randn(cout, device=dev)
    if not bwd:
        return t_(lambda: ops.head_fwd(x, pf, cout, b, g)), flop
    dyf = torch.randn((n, s, s, s, cout), device=dev)
    db = torch.empty(cout, device=dev)
    return t_(lambda: ops.head_bwd(dyf, pd, cin, dbias=db)), flop


def _head_loss(fused, n=2, s=96, cin=32, C=16):
    """the loss backward + the head's data gradient: partial_loss_bwd then head_bwd, or u3d_head_loss_bwd"""
    x, pf, pd, g, r, dy, flop = conv_case(n, cin, C, s, 1, 1, True)
    lg = torch.randn((n, s, s, s, C), device=dev)
    lab = torch.randint(0, C, (n, s, s, s), device=dev).float()
    wt = torch.ones(C, device=dev)
    _, sums = ops.partial_loss_fwd(lg, lab, wt)
    go = torch.ones(1, device=dev)
    db = torch.empty(C, device=dev)
    if fused:
        return t_(lambda: ops.head_loss_bwd(lg, lab, wt, sums, go, pd, cin, dbias=db)), flop
    return t_(lambda: ops.head_bwd(ops.partial_loss_bwd(lg, lab, wt, sums, go), pd, cin, dbias=db)), flop


def _small_step(s, dg, c=256, n=2):
    """the step's forms of the small-volume conv (12^3 / 6^3): forward + output statistics (+ residual), data gradient
    + GroupNorm-backward partials and finalize"""
    x, pf, pd, g, r, dy, flop = conv_case(n, c, c, s, 3, 1, True, not dg)
    if not dg:
        return t_(lambda: ops.conv_fwd_stats(x, pf, c, 3, 1, g, r)), flop
    dgam, dbet = torch.empty(c, device=dev), torch.empty(c, device=dev)
    return t_(lambda: ops.conv_dgrad_gn(dy, pd, c, x, 3, 1, g, dgb=lambda: (dgam, dbet))), flop


for s_ in (12, 6):
    CASES[f"fwd{s_}st"] = (lambda s_=s_: _small_step(s_, False))
    CASES[f"dgrad{s_}gb"] = (lambda s_=s_: _small_step(s_, True))
CASES["headloss96"] = lambda: _head_loss(True)
CASES["headloss96_2pass"] = lambda: _head_loss(False)
CASES["headf96"] = lambda: _head(False)
CASES["headb96"] = lambda: _head(True)
CASES["stemw96"] = lambda: _stemw()
CASES["loss96"] = lambda: _loss(2, 96, 16, False)
CASES["lossb96"] = lambda: _loss(2, 96, 16, True)


if __name__ == "__main__":
    names = sys.argv[1:] or list(CASES)
    for nm in names:
        us, flop = CASES[nm]()
        print(f"{nm:14s} {us:9.1f} us  {flop / us / 1e6:8.1f} TFLOP/s", flush=True)