"""Tensor-level wrappers over the libu3d C ABI. Torch is only the allocator / stream provider here: every
value is computed by a HIP kernel. All activations are NDHWC tensors of shape [n, d, h, w, c]."""
import contextlib
import ctypes
import os

import torch

from . import _lib
from ._lib import BF16, F32, call, query



def get_option(name):
    """Current value of a library tuning option (csrc/common.h ``Opt``)."""
    h = _lib.lib()
    if not hasattr(h, "u3d_get_option"):  # an A/B build of a tree older than the option table (U3D_LIB)
        return int(os.environ.get("U3D_" + name, {"CONVG_PERSIST": 1}.get(name, 0)))
    v = ctypes.c_int(0)
    if h.u3d_get_option(name.encode(), ctypes.byref(v)) != 0:
        raise _lib.U3DError(h.u3d_last_error().decode())
    return v.value


@contextlib.contextmanager
def option(name, value):
    """Temporarily set a library tuning option (csrc/common.h ``Opt``; e.g. ``option("CONVG_PERSIST", 0)``) for a test
    that compares two routings in one process; restores the previous value."""
    h = _lib.lib()
    if not hasattr(h, "u3d_set_option"):
        raise _lib.U3DError(f"u3d: this libu3d build has no option table (cannot set {name})")
    old = get_option(name)

    def put(v):
        if h.u3d_set_option(name.encode(), int(v)) != 0:
            raise _lib.U3DError(h.u3d_last_error().decode())
    put(value)
    try:
        yield
    finally:
        put(old)

def _ptr(t):
    return None if t is None else t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GET_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """torch's current HIP stream on the current device (the capture stream during graph capture). The direct C
    accessors: torch.cuda.current_stream().cuda_stream costs ~175 x 3-9 us of host time per training step (device
    index lookups, environment reads), which the eager step pays on its critical path (r04 host profile)."""
    if _RAW_STREAM is not None and _GET_DEVICE is not None:
        return _RAW_STREAM(_GET_DEVICE())
    return torch.cuda.current_stream().cuda_stream


def dt_code(dtype):
    if dtype == torch.float32:
        return F32
    if dtype == torch.bfloat16:
        return BF16
    raise _lib.U3DError(f"u3d: unsupported dtype {dtype}")


def require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.U3DError("u3d: the HIP path needs ROCm device tensors (no CPU fallback; the CPU "
                                "restatement lives in oracle/ and is test-only)")


def round32(c):
    return (c + 31) // 32 * 32


def out_dim(d, k, s):
    return (d + 2 * (k // 2) - k) // s + 1


class _WS:
    """Grow-only per-device scratch buffer (device memory owned by torch's caching allocator). Zero-filled when
    (re)allocated: the GroupNorm kernels keep completion counters at the head of their workspace and leave
    them at zero after every launch."""

    def __init__(self):
        self.buf = {}

    def get(self, nbytes, device, slot=0):
        key = (device, slot)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b


WS = _WS()


# ------------------------------------------------------------------------------------------ weights
def wstd_fwd(w, dtype, standardize=True, need_dgrad=True):
    """Standardise (unet3D.py:21-26) and pack a [cout, cin, k, k, k] fp32 weight."""
    require_device(w)
    cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
    k3 = k * k * k
    pf = torch.empty((k3, round32(cout), round32(cin)), dtype=dtype, device=w.device)
    pd = torch.empty((k3, round32(cin), round32(cout)), dtype=dtype, device=w.device) if need_dgrad else None
    st = torch.empty((cout, 2), dtype=torch.float32, device=w.device) if standardize else None
    call("u3d_wstd_fwd", dt_code(dtype), w.data_ptr(), cout, cin, k, int(standardize), pf.data_ptr(), _ptr(pd),
         _ptr(st), _stream())
    return pf, pd, st


WEIGHT_GEN = [0]     # bumped by every native in-place weight update (u3d.optim.SGD, DDP init broadcast)
_PACK_CACHE = {}     # inference only: standardised packs keyed by (weights, their versions, WEIGHT_GEN)
PACK_CACHE_OK = [os.environ.get("U3D_PACK_CACHE", "1") != "0"]  # off once an optimizer step is graph-captured


def _pack_key(items, dtype):
    return (dtype, WEIGHT_GEN[0], tuple((w.data_ptr(), w._version, tuple(w.shape), bool(s), bool(d))
                                        for w, s, d in items))


def wstd_fwd_batch(items, dtype):
    """Batched wstd_fwd over [(w, standardize, need_dgrad)]: one launch per 48 convs; packs and stats are
    views of three flat buffers. Returns [(pf, pd, st)] in item order. Under no_grad (inference, e.g. the 80
    sliding-window tiles of one volume) the packs of unchanged weights are reused: the key holds every weight's
    pointer and autograd version plus WEIGHT_GEN, which the native in-place updates bump."""
    if not items:
        return []
    if not torch.is_grad_enabled() and PACK_CACHE_OK[0] and not torch.cuda.is_current_stream_capturing():
        key = _pack_key(items, dtype)
        hit = _PACK_CACHE.get(key)
        if hit is not None:
            return hit
        out = _wstd_fwd_batch(items, dtype)
        if len(_PACK_CACHE) >= 4:
            _PACK_CACHE.clear()
        _PACK_CACHE[key] = out
        return out
    return _wstd_fwd_batch(items, dtype)


def _wstd_fwd_batch(items, dtype):
    dev = items[0][0].device
    shp = []
    nf = ns = 0
    for w, std, nd in items:
        require_device(w)
        cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
        n = k ** 3 * round32(cout) * round32(cin)
        shp.append((cout, cin, k, n))
        nf += n * (2 if nd else 1)
        ns += 2 * cout if std else 0
    buf = torch.empty((nf,), dtype=dtype, device=dev)
    sbuf = torch.empty((max(ns, 1),), dtype=torch.float32, device=dev)
    out, descs = [], []
    of = os_ = 0
    for (w, std, nd), (cout, cin, k, n) in zip(items, shp):
        pf = buf[of:of + n].view(k ** 3, round32(cout), round32(cin))
        of += n
        pd = None
        if nd:
            pd = buf[of:of + n].view(k ** 3, round32(cin), round32(cout))
            of += n
        st = None
        if std:
            st = sbuf[os_:os_ + 2 * cout].view(cout, 2)
            os_ += 2 * cout
        out.append((pf, pd, st))
        descs.append(_lib.WstdDesc(w.data_ptr(), pf.data_ptr(), _ptr(pd), _ptr(st), None, None, cout, cin, k,
                                   int(std), 1, 0))
    for i in range(0, len(descs), _lib.WSTD_BATCH_MAX):
        chunk = descs[i:i + _lib.WSTD_BATCH_MAX]
        arr = (_lib.WstdDesc * len(chunk))(*chunk)
        call("u3d_wstd_fwd_batch", dt_code(dtype), ctypes.addressof(arr), len(chunk), _stream())
    return out


def wstd_bwd_batch(items):
    """Batched wstd_bwd over [(partials, nsplit, w, wstats, standardize, dw, accumulate)]."""
    descs = [_lib.WstdDesc(w.data_ptr(), None, None, _ptr(st), part.data_ptr(), dw.data_ptr(), w.shape[0],
                           w.shape[1], w.shape[2], int(std), ns, int(acc))
             for part, ns, w, st, std, dw, acc in items]
    if not descs:
        return
    dev = items[0][2].device
    for i in range(0, len(descs), _lib.WSTD_BATCH_MAX):
        chunk = descs[i:i + _lib.WSTD_BATCH_MAX]
        arr = (_lib.WstdDesc * len(chunk))(*chunk)
        ws = WS.get(query("u3d_wstd_bwd_scratch_bytes", ctypes.addressof(arr), len(chunk)), dev, slot=5)
        call("u3d_wstd_bwd_batch", ctypes.addressof(arr), len(chunk), ws.data_ptr(), _stream())


def wstd_bwd(partials, nsplit, w, wstats, standardize, dw=None, accumulate=False):
    cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
    if dw is None:
        dw = torch.empty_like(w)
        accumulate = False
    call("u3d_wstd_bwd", partials.data_ptr(), nsplit, w.data_ptr(), _ptr(wstats), cout, cin, k, int(standardize),
         dw.data_ptr(), int(accumulate), _stream())
    return dw


# ------------------------------------------------------------------------------------------ convs
# bf16 1^3 convs (stride 1 / 2, GN prologue in registers) and stride-1 1^3 data gradients: streaming kernel
# (conv1x1.hip) instead of the implicit GEMM (+ GN materialisation). U3D_CONV1X1=0: the implicit GEMM.
USE_CONV1X1 = os.environ.get("U3D_CONV1X1", "1") != "0"


def _use_conv1x1(dtype, cx, cy, k, n):
    return USE_CONV1X1 and k == 1 and dtype == torch.bfloat16 and cx % 8 == 0 and cy % 8 == 0 and max(cx, cy) <= 256 \
        and n <= 65535


def conv_fwd(x, wpk, cout, k, stride, gn=None, residual=None, bias=None, out_f32=False):
    """x: [n,d,h,w,cin] -> [n,od,oh,ow,cout]. gn = (stats, gamma, beta, groups) fuses GroupNorm+ReLU."""
    require_device(x)
    n, d, h, w_, cin = x.shape
    od, oh, ow = out_dim(d, k, stride), out_dim(h, k, stride), out_dim(w_, k, stride)
    y = torch.empty((n, od, oh, ow, cout), dtype=torch.float32 if out_f32 else x.dtype, device=x.device)
    st, ga, be, G = gn if gn is not None else (None, None, None, 0)
    if _use_conv1x1(x.dtype, cin, cout, k, n) and residual is None and bias is None and not out_f32:
        call("u3d_conv1x1", x.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), wpk.shape[-1], cout, stride, _ptr(st),
             _ptr(ga), _ptr(be), G, y.data_ptr(), _stream())
        return y
    if _use_conv32(x.dtype, cin, cout, k, stride, n, w_) and _conv32_fits(x) and not out_f32 and bias is None:
        pr = _probe0()
        if _ring_queue():
            call("u3d_conv32_ring_q", 0, x.data_ptr(), n, d, h, w_, wpk.data_ptr(), _ptr(st), _ptr(ga), _ptr(be), G,
                 _ptr(residual), y.data_ptr(), None, _queue(x.device, (n, d, h, w_)), _stream())
        else:
            call(CONV32_FN, 0, x.data_ptr(), n, d, h, w_, wpk.data_ptr(), _ptr(st), _ptr(ga), _ptr(be), G,
                 _ptr(residual), y.data_ptr(), _stream())
        _probe1(pr, "conv32_ring fwd" + (" GN" if st is not None else "") + (" +res" if residual is not None else ""),
                2.0 * n * d * h * w_ * 27 * 32 * 32, n * d * h * w_)
        return y
    if _use_small(x.dtype, cin, cout, k, stride, (n, d, h, w_)) and not out_f32 and bias is None:
        conv_small(0, x, cin, wpk, cout, (st, ga, be, G), residual, y)
        return y
    if _use_gen_brick(x.dtype, cin, cout, k, stride, (n, d, h, w_)) and not out_f32 and bias is None:
        call("u3d_convg_brick", 0, x.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), cout, _ptr(st), _ptr(ga), _ptr(be),
             G, _ptr(residual), y.data_ptr(), _stream())
        return y
    if (st is not None and x.dtype == torch.bfloat16 and cin >= GN_MATERIALIZE_MIN_C
            and x.numel() * 2 <= GN_MATERIALIZE_BYTES):
        # small deep-layer activation: materialise relu(gn(x)) once so the GEMM K loop has no GN arithmetic
        x = gn_apply(x, st, ga, be, G)
        st = ga = be = None
        G = 0
    ws = WS.get(SPLITK_WS_BYTES, x.device, slot=4)
    call("u3d_conv_fwd", dt_code(x.dtype), x.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), cout, k, stride, _ptr(st),
         _ptr(ga), _ptr(be), G, _ptr(residual), _ptr(bias), y.data_ptr(), int(out_f32), ws.data_ptr(), ws.numel(),
         _stream())
    return y


# conv_small's split-K slabs combined inside its launch by each output tile's last-arriving workgroup (round 5,
# u3d_conv_small2: no small_reduce_kernel launch); U3D_SMALL_FUSE=0: the two-kernel form
SMALL_FUSE = os.environ.get("U3D_SMALL_FUSE", "1") != "0"
SMALL_CNT_SLOT, SMALL_SPART_SLOT = 16, 17


def conv_small(flip, x, cin, wpk, cout, gn, residual, y, want_stats=False):
    """u3d_conv_small(2) into y; returns the output's GroupNorm(16) statistics [n,16,2] when want_stats and the launch
    produced them (in-kernel combine with the contraction split), else None."""
    n, d, h, w_ = x.shape[:4]
    st, ga, be, G = gn if gn is not None else (None, None, None, 0)
    ws = WS.get(SPLITK_WS_BYTES, x.device, slot=4)
    if not SMALL_FUSE:
        call("u3d_conv_small", flip, x.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), cout, _ptr(st), _ptr(ga),
             _ptr(be), G, _ptr(residual), y.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        return None
    cnt = WS.get(query("u3d_conv_small_cnt_bytes", n, d, h, w_, cout), x.device, slot=SMALL_CNT_SLOT)
    stats = sp = None
    if want_stats:
        stats = torch.empty((n, 16, 2), dtype=torch.float32, device=x.device)
        sp = WS.get(4 * query("u3d_conv_small_spart_floats", n, d, h, w_), x.device, slot=SMALL_SPART_SLOT)
    made = ctypes.c_int(0)
    call("u3d_conv_small2", flip, x.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), cout, _ptr(st), _ptr(ga), _ptr(be),
         G, _ptr(residual), y.data_ptr(), ws.data_ptr(), ws.numel(), cnt.data_ptr(), _ptr(sp), _ptr(stats),
         ctypes.addressof(made), _stream())
    return stats if made.value else None


# the forward ring stores relu(gn(x)) for the weight gradient (round 6; measured slower, off: the forward rings pay
# +16-19 us per launch for the side stores, the GN-free weight gradient saves 7.5 us per launch; step 5.76 vs 5.62 ms)
RING_XN = os.environ.get("U3D_RING_XN", "0") != "0"


def ring_xn_ok(x, cout, k, stride, gn):
    """Whether conv_fwd_stats_xn applies: the static 32->32 ring forward with its GroupNorm prologue (bf16)."""
    n, d, h, w_, cin = x.shape
    return (RING_XN and RING_STATS and gn is not None and cout == 32 and CONV32_FN == "u3d_conv32_ring"
            and not FUSED_FINALIZE and not _ring_queue() and _use_conv32(x.dtype, cin, cout, k, stride, n, w_)
            and _conv32_fits(x))


# stride-2 3^3 convs with cin >= 64 (the 48^3 / 24^3 / 12^3 downsampling convs on the implicit GEMM): normalise the
# input once (round 6, kbench gpurun_out/r06_g: 48^3 forward 65.5 -> 48.4 + 14.1 us, its weight gradient 36.0 -> 30.2)
S2_NORM_ONCE = os.environ.get("U3D_S2_NORM_ONCE", "1") != "0"


def s2_normalise_once(x, cin, cout, k, stride, gn):
    return (S2_NORM_ONCE and gn is not None and k == 3 and stride == 2 and x.dtype == torch.bfloat16 and cin >= 64
            and cin % 8 == 0 and not (S2_RING and cin == 32 and cout == 64))


def conv_fwd_stats_xn(x, wpk, cout, k, stride, gn, residual=None):
    """conv_fwd_stats on the static ring that also returns xn = relu(gn(x)) (bf16 NDHWC, x's shape), stored by the
    ring from its staged input: the conv's weight gradient then reads xn without a GroupNorm prologue (bitwise the
    same partials as conv_wgrad(dy, x, ..., gn)). Caller checks ring_xn_ok. Returns (y, stats, xn)."""
    n, d, h, w_, cin = x.shape
    st, ga, be, G = gn
    y = torch.empty((n, d, h, w_, cout), dtype=x.dtype, device=x.device)
    xn = torch.empty_like(x)
    stats = torch.empty((n, 16, 2), dtype=torch.float32, device=x.device)
    ws = WS.get(4 * query("u3d_conv32_ring_stats_ws_floats", n), x.device, slot=9)
    pr = _probe0()
    call("u3d_conv32_ring_stats_xn", x.data_ptr(), n, d, h, w_, wpk.data_ptr(), st.data_ptr(), ga.data_ptr(),
         be.data_ptr(), G, _ptr(residual), y.data_ptr(), xn.data_ptr(), ws.data_ptr(), _stream())
    _probe1(pr, "conv32_ring fwd GN" + (" +res" if residual is not None else "") + " +stats",
            2.0 * n * d * h * w_ * 27 * 32 * 32, n * d * h * w_)
    call("u3d_conv32_ring_stats_finalize", ws.data_ptr(), n, d, h, w_, stats.data_ptr(), _stream())
    return y, stats, xn


def conv_fwd_stats(x, wpk, cout, k, stride, gn=None, residual=None):
    """conv_fwd that also returns the GroupNorm(16) statistics [n,16,2] of its output when the 32->32 ring kernel
    runs with a GN prologue (epilogue-accumulated); otherwise (conv_fwd(...), None)."""
    n, d, h, w_, cin = x.shape
    if (RING_STATS and gn is not None and cout == 32 and CONV32_FN == "u3d_conv32_ring"
            and _use_conv32(x.dtype, cin, cout, k, stride, n, w_) and _conv32_fits(x)):
        st, ga, be, G = gn
        y = torch.empty((n, d, h, w_, cout), dtype=x.dtype, device=x.device)
        stats = torch.empty((n, 16, 2), dtype=torch.float32, device=x.device)
        q = _ring_queue()
        nws = query("u3d_conv32_ring_q_stats_ws_floats", n, d, h, w_) if q else query("u3d_conv32_ring_stats_ws_floats", n)
        ws = WS.get(4 * nws, x.device, slot=9)
        pr = _probe0()
        if q:
            call("u3d_conv32_ring_q", 0, x.data_ptr(), n, d, h, w_, wpk.data_ptr(), st.data_ptr(), ga.data_ptr(),
                 be.data_ptr(), G, _ptr(residual), y.data_ptr(), ws.data_ptr(), _queue(x.device, (n, d, h, w_)), _stream())
        elif FUSED_FINALIZE:  # the statistics finalized by the launch's last-arriving workgroup (round 5)
            call("u3d_conv32_ring_stats_fused", x.data_ptr(), n, d, h, w_, wpk.data_ptr(), st.data_ptr(), ga.data_ptr(),
                 be.data_ptr(), G, _ptr(residual), y.data_ptr(), ws.data_ptr(), stats.data_ptr(),
                 WS.get(256, x.device, slot=RING_CNT_SLOT).data_ptr(), _stream())
        else:
            call("u3d_conv32_ring_stats", x.data_ptr(), n, d, h, w_, wpk.data_ptr(), st.data_ptr(), ga.data_ptr(),
                 be.data_ptr(), G, _ptr(residual), y.data_ptr(), ws.data_ptr(), _stream())
        _probe1(pr, "conv32_ring fwd GN" + (" +res" if residual is not None else "") + " +stats",
                2.0 * n * d * h * w_ * 27 * 32 * 32, n * d * h * w_)
        if q or not FUSED_FINALIZE:
            fin = "u3d_conv32_ring_q_stats_finalize" if q else "u3d_conv32_ring_stats_finalize"
            call(fin, ws.data_ptr(), n, d, h, w_, stats.data_ptr(), _stream())
        return y, stats
    if (S2_RING and gn is not None and residual is None and k == 3 and stride == 2 and x.dtype == torch.bfloat16
            and cin == 32 and cout == 64 and query("u3d_conv_s2_ring_ok", n, cin, d, h, w_, cout)):
        # stride-2 forward as an input-plane walk, GN applied once per staged element, output statistics in-kernel
        st, ga, be, G = gn
        od, oh, ow = out_dim(d, 3, 2), out_dim(h, 3, 2), out_dim(w_, 3, 2)
        y = torch.empty((n, od, oh, ow, cout), dtype=x.dtype, device=x.device)
        stats = torch.empty((n, 16, 2), dtype=torch.float32, device=x.device)
        sp = WS.get(4 * query("u3d_conv_s2_ring_ws_floats", n, d, h, w_), x.device, slot=S2_SPART_SLOT)
        call("u3d_conv_s2_ring", x.data_ptr(), n, d, h, w_, wpk.data_ptr(), st.data_ptr(), ga.data_ptr(), be.data_ptr(),
             G, y.data_ptr(), sp.data_ptr(), stats.data_ptr(), WS.get(256, x.device, slot=S2_CNT_SLOT).data_ptr(),
             _stream())
        return y, stats
    if (SMALL_FUSE and SMALL_STATS and cout in (64, 128, 256) and _use_small(x.dtype, cin, cout, k, stride, (n, d, h, w_))
            and not _use_conv1x1(x.dtype, cin, cout, k, n) and not _use_conv32(x.dtype, cin, cout, k, stride, n, w_)):
        y = torch.empty((n, d, h, w_, cout), dtype=x.dtype, device=x.device)
        stats = conv_small(0, x, cin, wpk, cout, gn, residual, y, want_stats=True)
        if stats is not None:
            return y, stats
        return y, None
    if (BRICK_STATS and cout % 32 == 0 and cin <= 256 and k == 3 and stride == 1
            and _use_gen_brick(x.dtype, cin, cout, k, stride, (n, d, h, w_))
            and not _use_conv1x1(x.dtype, cin, cout, k, n) and not _use_conv32(x.dtype, cin, cout, k, stride, n, w_)
            and not _use_small(x.dtype, cin, cout, k, stride, (n, d, h, w_))
            and get_option("CONVG_PERSIST") != 0):
        # persistent brick conv with the output's GroupNorm(16) statistics from its epilogue (no statistics pass)
        st, ga, be, G = gn if gn is not None else (None, None, None, 0)
        y = torch.empty((n, d, h, w_, cout), dtype=x.dtype, device=x.device)
        stats = torch.empty((n, 16, 2), dtype=torch.float32, device=x.device)
        nws = query("u3d_convg_brick_stats_ws_floats", n, d, h, w_, cout)
        ws = WS.get(4 * nws, x.device, slot=9)
        if FUSED_FINALIZE:
            call("u3d_convg_brick_stats_fused", x.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), cout, _ptr(st), _ptr(ga),
                 _ptr(be), G, _ptr(residual), y.data_ptr(), ws.data_ptr(), nws, stats.data_ptr(),
                 WS.get(256, x.device, slot=BRICK_CNT_SLOT).data_ptr(), _stream())
        else:
            call("u3d_convg_brick_stats", x.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), cout, _ptr(st), _ptr(ga),
                 _ptr(be), G, _ptr(residual), y.data_ptr(), ws.data_ptr(), nws, stats.data_ptr(), _stream())
        return y, stats
    return conv_fwd(x, wpk, cout, k, stride, gn, residual), None


# Work-stealing ring (u3d_conv32_ring_q): robust to a concurrent kernel holding CUs (a late workgroup's range is
# taken over by the others instead of doubling the launch), but 10-25% slower alone (tools/concurrency.py,
# profiles/r02_concurrency.json), and its GroupNorm backward takes the separate partial pass (another fp32 order
# than the fused static ring). Used for the data-gradient ring only while COLLECTIVE_IN_FLIGHT is set;
# U3D_RING_QUEUE=1 forces it for every ring launch.
RING_QUEUE = os.environ.get("U3D_RING_QUEUE", "0") != "0"
# The collective-tolerant forms (work-stealing data-gradient ring, short-range weight-gradient ring) are chosen
# STATICALLY, never from a device poll, so a data-parallel step runs the same kernels and produces the same bits
# every time. Default (DDP_TOLERANT off): the data-parallel backward runs exactly the plain step's forms, so an N-rank
# step is bitwise the 1-rank step up to the all-reduce itself. U3D_DDP_TOLERANT=1: the tolerant forms from the first
# bucket launch of a backward to its end (a latch in tape order: deterministic, but other fp32 sums than the plain
# step's GroupNorm backward).
DDP_TOLERANT = [os.environ.get("U3D_DDP_TOLERANT", "0") != "0"]
COLLECTIVE_IN_FLIGHT = [False]  # the latch: set by u3d.ddp at a bucket launch when DDP_TOLERANT (tests may set it)


def collective_in_flight():
    """Whether the collective-tolerant kernel forms run now (a static latch, see DDP_TOLERANT)."""
    return COLLECTIVE_IN_FLIGHT[0]


def _ring_queue(dgrad=False):
    return CONV32_FN == "u3d_conv32_ring" and (RING_QUEUE or (dgrad and collective_in_flight()))


QUEUE_SLOT = 40  # workspace slot of the ring claim words (used by nothing else: the words must stay zero between launches)


def _queue(device, shape):
    """Zeroed claim words for the work-stealing ring kernels (left zero by every launch; one queue: launches are
    stream-ordered on the caller's stream)."""
    return WS.get(query("u3d_conv32_ring_q_queue_bytes", *shape), device, slot=QUEUE_SLOT).data_ptr()


# the ring / persistent-brick conv epilogue statistics (and the ring data gradient's GroupNorm-backward coefficients)
# finalized by the conv launch's last-arriving workgroup instead of a separate finalize launch (round 5, U3D_FUSED_FINALIZE=1).
# Off by default: measured no cheaper than the launch it replaces (step A/B r05_e 5.671 / 5.672 off vs 5.687 / 5.678 on;
# the in-step ring / brick launches grow 4-8 us each by the last arriver's drain + atomic + cross-XCD loads, r05_f trace)
FUSED_FINALIZE = os.environ.get("U3D_FUSED_FINALIZE", "0") != "0"
RING_CNT_SLOT, BRICK_CNT_SLOT, RING_GB_CNT_SLOT = 18, 19, 23
# the 96^3 stride-2 3^3 forward (cin 32 -> cout 64, GN prologue) as an input-plane walk (conv_s2.hip, round 5);
# U3D_S2_RING=0: the implicit GEMM + a statistics pass
S2_RING = os.environ.get("U3D_S2_RING", "1") != "0"
S2_SPART_SLOT, S2_CNT_SLOT = 21, 22
SMALL_STATS = os.environ.get("U3D_SMALL_STATS", "1") != "0"  # GN(16) stats of conv_small outputs from its combine
BRICK_STATS = os.environ.get("U3D_BRICK_STATS", "1") != "0"  # GN statistics from the persistent brick's epilogue
RING_STATS = os.environ.get("U3D_RING_STATS", "1") != "0"  # GroupNorm statistics from the ring conv epilogue (False: separate u3d_gn_stats pass)
SPLITK_WS_BYTES = 64 << 20
# bench.py roofline: while PROBE is a list, every launch of the 96^3-class ring kernels (conv fwd / dgrad and the
# stride-1 weight-gradient ring) records (start event, end event, label, flop, voxels) on the stream it runs on
PROBE = None


def _probe0():
    if PROBE is None:
        return None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    return e0, e1


def _probe1(p, label, flop, vox):
    if p is not None:
        p[1].record()
        PROBE.append((p[0], p[1], label, flop, vox))
USE_CONV32_BRICK = True
CONV32_FN = "u3d_conv32_ring"   # "u3d_conv32_brick": the earlier halo-brick schedule (same results)


def _use_conv32(dtype, cin, cout, k, stride, n, w=32):
    if not (USE_CONV32_BRICK and dtype == torch.bfloat16 and cin == 32 and cout == 32 and k == 3 and stride == 1):
        return False
    return CONV32_FN == "u3d_conv32_ring" or (n <= 16 and w % 32 == 0)


def _conv32_fits(x):
    return CONV32_FN != "u3d_conv32_ring" or x.numel() * x.element_size() < (1 << 31)  # 32-bit buffer offsets


USE_SMALL_CONV = True
SMALL_MAX_VOX = 2 * 12 ** 3  # n*d*h*w up to which the small-volume brick kernel (conv_small.hip) runs (24^3: convg)


def _use_small(dtype, cin, cout, k, stride, shape):
    n, d, h, w_ = shape
    return USE_SMALL_CONV and dtype == torch.bfloat16 and k == 3 and stride == 1 and cin % 8 == 0 \
        and cout % 8 == 0 and n * d * h * w_ <= SMALL_MAX_VOX


USE_GEN_BRICK = True
BRICK_MIN_WG = 128  # below this many workgroups the split-K implicit GEMM fills the chip better


def _use_gen_brick(dtype, cin, cout, k, stride, shape):
    if not (USE_GEN_BRICK and dtype == torch.bfloat16 and k == 3 and stride == 1 and cin % 8 == 0 and cout % 8 == 0):
        return False
    n, d, h, w_ = shape
    if n > 16:
        return False
    nb = n * -(-d // 4) * -(-h // 8) * -(-w_ // 16)
    # workgroups with 64-channel co tiles, or with 32-channel ones (the launcher picks those when 64 give too few)
    return max(nb * max(1, -(-cout // 64)), nb * max(1, -(-cout // 32))) >= BRICK_MIN_WG


GN_BWD_FUSED = os.environ.get("U3D_GN_BWD_FUSED", "1") != "0"  # GroupNorm-backward partials in the ring dgrad epilogue


def conv_dgrad_gn(dy, wpk_dgrad, cin, x, k, stride, gn, dgb=None):
    """Data gradient of conv(relu(gn(x))) with the GroupNorm backward's partial pass fused into the ring epilogue
    (u3d_conv32_ring_dgrad_gn): returns (dA, parts) for gn_bwd_parts, or None where the static 32-channel ring does
    not run this conv (the caller then takes conv_dgrad + gn_bwd). On the small-volume kernel (and with ``dgb``, a
    callable returning the (dgamma, dbeta) destinations) the finalize runs inside the launch too: parts is then
    ("coef", coef) for gn_bwd_apply_coef, dgamma / dbeta already written."""
    n, d, h, w_ = x.shape[:4]
    if not (GN_BWD_FUSED and gn is not None and dy.shape[-1] == 32 and _use_conv32(dy.dtype, cin, 32, k, stride, n, w_)
            and CONV32_FN == "u3d_conv32_ring" and _conv32_fits(dy) and not _ring_queue(dgrad=True)):
        if dgb is not None:
            r = _conv_dgrad_gn_small(dy, wpk_dgrad, cin, x, k, stride, gn, dgb)
            if r is not None:
                return r
        return _conv_dgrad_gn_brick(dy, wpk_dgrad, cin, x, k, stride, gn)
    st, ga, be, G = gn
    wps = query("u3d_conv32_ring_wps", n, d, h, w_)
    da = torch.empty((n, d, h, w_, cin), dtype=dy.dtype, device=dy.device)
    parts = torch.empty((n, wps, 32, 2), dtype=torch.float32, device=dy.device)
    pr = _probe0()
    if FUSED_FINALIZE and dgb is not None:  # the finalize by the launch's last-arriving workgroup (round 5)
        dg, db = dgb()
        coef = torch.empty((n, 5, 32), dtype=torch.float32, device=dy.device)
        call("u3d_conv32_ring_dgrad_gn_fused", dy.data_ptr(), n, d, h, w_, wpk_dgrad.data_ptr(), x.data_ptr(),
             st.data_ptr(), ga.data_ptr(), be.data_ptr(), G, da.data_ptr(), parts.data_ptr(), coef.data_ptr(), _ptr(dg),
             _ptr(db), WS.get(256, dy.device, slot=RING_GB_CNT_SLOT).data_ptr(), _stream())
        _probe1(pr, "conv32_ring dgrad +GN-bwd partials", 2.0 * n * d * h * w_ * 27 * 32 * 32, n * d * h * w_)
        return da, ("coef", coef)
    call("u3d_conv32_ring_dgrad_gn", dy.data_ptr(), n, d, h, w_, wpk_dgrad.data_ptr(), x.data_ptr(), st.data_ptr(),
         ga.data_ptr(), be.data_ptr(), G, da.data_ptr(), parts.data_ptr(), _stream())
    _probe1(pr, "conv32_ring dgrad +GN-bwd partials", 2.0 * n * d * h * w_ * 27 * 32 * 32, n * d * h * w_)
    return da, parts


GN_BWD_FUSED_BRICK = os.environ.get("U3D_GN_BWD_FUSED_BRICK", "1") != "0"  # the same in the persistent brick
# ... up to this many voxels (n*d*h*w): the fused epilogue pays where the separate partial pass is latency-bound. Kernel
# A/B (tools/kbench.py gnb*, gpurun_out/r04_g): 2x24^3 x 128 ch 51.4 -> 47.9 us for the data gradient + GN backward,
# 2x48^3 x 64 ch 89.7 -> 92.5 us (the x loads and the epilogue sums outweigh the 56 MB partial pass there)
GN_BWD_FUSED_BRICK_MAX_VOX = int(os.environ.get("U3D_GN_BWD_FUSED_BRICK_MAX_VOX", str(2 * 32 ** 3)))


SMALL_GB = os.environ.get("U3D_SMALL_GB", "1") != "0"  # GN-backward partials + finalize in the small-volume dgrad


def _conv_dgrad_gn_small(dy, wpk_dgrad, cin, x, k, stride, gn, dgb):
    """conv_dgrad_gn where conv_dgrad would run the small-volume kernel (u3d_conv_small_dgrad_gn): the partial pass and
    the coefficient finalize inside the data-gradient launch; returns (dA, ("coef", coef)) or None."""
    shape = tuple(x.shape[:4])
    n, d, h, w_ = shape
    cout = dy.shape[-1]
    if not (GN_BWD_FUSED and SMALL_GB and SMALL_FUSE and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
            and k == 3 and stride == 1 and _use_small(dy.dtype, cout, cin, k, stride, shape) and cin % 8 == 0
            and n * cin * 2 <= 8192):
        return None
    st, ga, be, G = gn
    dg, db = dgb()
    da = torch.empty((n, d, h, w_, cin), dtype=dy.dtype, device=dy.device)
    coef = torch.empty((n, 5, cin), dtype=torch.float32, device=dy.device)
    ws = WS.get(SPLITK_WS_BYTES, dy.device, slot=4)
    cnt = WS.get(query("u3d_conv_small_cnt_bytes", n, d, h, w_, cin), dy.device, slot=SMALL_CNT_SLOT)
    parts = WS.get(4 * query("u3d_conv_small_gb_parts_floats", n, d, h, w_, cin), dy.device, slot=SMALL_GB_SLOT)
    made = ctypes.c_int(0)
    call("u3d_conv_small_dgrad_gn", dy.data_ptr(), n, cout, d, h, w_, wpk_dgrad.data_ptr(), cin, x.data_ptr(),
         st.data_ptr(), ga.data_ptr(), be.data_ptr(), G, da.data_ptr(), ws.data_ptr(), ws.numel(), cnt.data_ptr(),
         parts.data_ptr(), coef.data_ptr(), _ptr(dg), _ptr(db), ctypes.addressof(made), _stream())
    if not made.value:
        return None
    return da, ("coef", coef)


SMALL_GB_SLOT = 20


def gn_bwd_apply_coef(da, x, coef, groups, dx=None, accumulate=False):
    """The apply pass of the GroupNorm backward from precomputed coefficients (u3d_conv_small_dgrad_gn)."""
    n, c = x.shape[0], x.shape[-1]
    v = x.numel() // (n * c)
    if dx is None:
        dx = torch.empty_like(x)
        accumulate = False
    call("u3d_gn_bwd_apply_coef", da.data_ptr(), x.data_ptr(), n, c, v, groups, coef.data_ptr(), dx.data_ptr(),
         int(accumulate), _stream())
    return dx


def _conv_dgrad_gn_brick(dy, wpk_dgrad, cin, x, k, stride, gn):
    """conv_dgrad_gn where conv_dgrad would run the persistent brick (u3d_convg_brick_dgrad_gn): parts per brick."""
    if not (GN_BWD_FUSED and GN_BWD_FUSED_BRICK and gn is not None and dy.dtype == torch.bfloat16):
        return None
    shape = tuple(x.shape[:4])
    cout = dy.shape[-1]
    n, d, h, w_ = shape
    if n * d * h * w_ > GN_BWD_FUSED_BRICK_MAX_VOX:
        return None
    # only where conv_dgrad itself runs the generic brick (not the 32-channel ring, e.g. its queue form under a
    # collective, nor the small-volume kernel)
    if _use_conv32(dy.dtype, cin, cout, k, stride, n, w_) and _conv32_fits(dy):
        return None
    if _use_small(dy.dtype, cout, cin, k, stride, shape) or not _use_gen_brick(dy.dtype, cout, cin, k, stride, shape):
        return None
    nparts = query("u3d_convg_brick_gn_nparts", n, cin, d, h, w_, cout)
    if nparts <= 0:
        return None
    st, ga, be, G = gn
    da = torch.empty((n, d, h, w_, cin), dtype=dy.dtype, device=dy.device)
    parts = torch.empty((n, nparts, cin, 2), dtype=torch.float32, device=dy.device)
    call("u3d_convg_brick_dgrad_gn", dy.data_ptr(), n, cout, d, h, w_, wpk_dgrad.data_ptr(), cin, x.data_ptr(),
         st.data_ptr(), ga.data_ptr(), be.data_ptr(), G, da.data_ptr(), parts.data_ptr(), nparts, _stream())
    return da, parts


def conv_dgrad(dy, wpk_dgrad, cin, in_shape, k, stride):
    n, d, h, w_ = in_shape
    cout = dy.shape[-1]
    dx = torch.empty((n, d, h, w_, cin), dtype=dy.dtype, device=dy.device)
    if stride == 1 and _use_conv1x1(dy.dtype, cout, cin, k, n):  # dx = dy . W^T: the dgrad pack is [cin_p][cout_p]
        call("u3d_conv1x1", dy.data_ptr(), n, cout, d, h, w_, wpk_dgrad.data_ptr(), wpk_dgrad.shape[-1], cin, 1, None,
             None, None, 0, dx.data_ptr(), _stream())
        return dx
    if _use_conv32(dy.dtype, cin, cout, k, stride, n, w_) and _conv32_fits(dy):
        pr = _probe0()
        q = _ring_queue(dgrad=True)
        if q:
            call("u3d_conv32_ring_q", 1, dy.data_ptr(), n, d, h, w_, wpk_dgrad.data_ptr(), None, None, None, 0, None,
                 dx.data_ptr(), None, _queue(dy.device, (n, d, h, w_)), _stream())
        else:
            call(CONV32_FN, 1, dy.data_ptr(), n, d, h, w_, wpk_dgrad.data_ptr(), None, None, None, 0, None,
                 dx.data_ptr(), _stream())
        _probe1(pr, "conv32_ring dgrad" + (" (work stealing)" if q else ""), 2.0 * n * d * h * w_ * 27 * 32 * 32,
                n * d * h * w_)
        return dx
    if (USE_S2_BRICK and dy.dtype == torch.bfloat16 and k == 3 and stride == 2
            and dy.numel() * dy.element_size() < (1 << 31) - 64):  # (its dy reads use 32-bit buffer offsets)
        call("u3d_conv_dgrad_s2", dy.data_ptr(), n, cout, wpk_dgrad.data_ptr(), cin, d, h, w_, dx.data_ptr(),
             _stream())
        return dx
    if _use_small(dy.dtype, cout, cin, k, stride, (n, d, h, w_)):
        conv_small(1, dy, cout, wpk_dgrad, cin, None, None, dx)
        return dx
    if _use_gen_brick(dy.dtype, cout, cin, k, stride, (n, d, h, w_)):
        call("u3d_convg_brick", 1, dy.data_ptr(), n, cout, d, h, w_, wpk_dgrad.data_ptr(), cin, None, None, None, 0,
             None, dx.data_ptr(), _stream())
        return dx
    ws = WS.get(SPLITK_WS_BYTES, dy.device, slot=4)
    call("u3d_conv_dgrad", dt_code(dy.dtype), dy.data_ptr(), n, cout, wpk_dgrad.data_ptr(), cin, d, h, w_, k, stride,
         dx.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
    return dx


# the downsample branch's stride-2 1^3 data gradient kept at the conv's output resolution when its GroupNorm backward
# runs paired with gn1 (gn_bwd2(..., da2_s2=True)): no zero-filled full-resolution tensor (U3D_S2_COMPACT=0: off)
S2_COMPACT = os.environ.get("U3D_S2_COMPACT", "1") != "0"


def s2_compact_ok(in_shape, cin, elsize):
    """Limits of the paired GroupNorm backward that reads a compact stride-2 1^3 data gradient (u3d_gn_bwd2_s2,
    groupnorm.hip: the voxel -> (z, y, x) split by an fp32 reciprocal needs < 2^24 voxels per sample; the compact
    operand is read with 32-bit buffer offsets, < 2 GiB). Outside them the caller takes conv_dgrad + gn_bwd2."""
    n, d, h, w_ = in_shape[:4]
    cv = out_dim(d, 1, 2) * out_dim(h, 1, 2) * out_dim(w_, 1, 2)
    return d * h * w_ < (1 << 24) and n * cv * cin * elsize < (1 << 31)


def conv_dgrad_1x1s2_compact(dy, wpk_dgrad, cin):
    """dx of a stride-2 1^3 conv at the conv's OUTPUT resolution (the values at the even input voxels; every
    other input voxel's gradient is zero)."""
    n, od, oh, ow, cout = dy.shape
    dxc = torch.empty((n, od, oh, ow, cin), dtype=dy.dtype, device=dy.device)
    call("u3d_conv1x1", dy.data_ptr(), n, cout, od, oh, ow, wpk_dgrad.data_ptr(), wpk_dgrad.shape[-1], cin, 1, None,
         None, None, 0, dxc.data_ptr(), _stream())
    return dxc


def expand_s2(dxc, in_shape):
    """Full-resolution tensor of a compact stride-2 1^3 data gradient (zeros at the odd voxels)."""
    n, d, h, w_ = in_shape
    full = torch.zeros((n, d, h, w_, dxc.shape[-1]), dtype=dxc.dtype, device=dxc.device)
    full[:, ::2, ::2, ::2] = dxc
    return full


USE_BRICK_WGRAD = True
USE_RING_WGRAD = True      # stride-1 3^3 weight gradients: depth-streaming ring kernel (wgrad_ring.hip)
RING_WGRAD_MIN_HW = 8      # h, w extents below this use the brick kernel (measured faster from 12^3 up)
USE_S2_BRICK = True  # stride-2 3^3 bf16 data gradient: one-launch parity-merged kernel (dgrad_s2.hip)
# stride-1 weight-gradient ring while a collective may hold CUs (or always with U3D_WGRAD_QUEUE=1): a grid of ~3x the
# CUs in short plane ranges instead of one resident range per CU (each range keeps its own slab: same sums every run)
WGRAD_QUEUE = os.environ.get("U3D_WGRAD_QUEUE", "0") != "0"
WGRAD_Q_WGS = 768


def conv_wgrad(dy, x, k, stride, gn=None, brick=None):
    """Returns (partials fp32 [nsplit, k^3, cout_p, cin_p], nsplit). bf16 3^3 convs use the halo-brick kernel."""
    n, d, h, w_, cin = x.shape
    cout = dy.shape[-1]
    st, ga, be, G = gn if gn is not None else (None, None, None, 0)
    if brick is None:
        brick = USE_BRICK_WGRAD and x.dtype == torch.bfloat16
        if (brick and k == 3 and stride == 1 and USE_RING_WGRAD and min(h, w_) >= RING_WGRAD_MIN_HW
                and max(x.numel() * x.element_size(), dy.numel() * dy.element_size()) < (1 << 31)):
            brick = "ring"  # (the ring addresses its operands with 32-bit buffer offsets; larger ones: bricks)
    if brick == "ring":
        assert k == 3 and stride == 1 and x.dtype == torch.bfloat16
        if WGRAD_QUEUE or collective_in_flight():  # short ranges the dispatcher deals to whichever CU is free
            ns = query("u3d_conv_wgrad_ring_splits_target", n, cin, d, h, w_, cout, WGRAD_Q_WGS)
        else:
            ns = query("u3d_conv_wgrad_ring_splits", n, cin, d, h, w_, cout)
        part = torch.empty((ns, 27, round32(cout), round32(cin)), dtype=torch.float32, device=x.device)
        pr = _probe0()
        call("u3d_conv_wgrad_ring", dy.data_ptr(), x.data_ptr(), n, cin, d, h, w_, cout, _ptr(st), _ptr(ga), _ptr(be),
             G, part.data_ptr(), ns, _stream())
        _probe1(pr, f"wgrad_ring {cin}->{cout}" + (" GN" if st is not None else ""),
                2.0 * n * d * h * w_ * 27 * cin * cout, n * d * h * w_)
        return part, ns
    if brick and k == 1:
        ns = query("u3d_conv_wgrad1_splits", n, cin, d, h, w_, cout, stride)
        part = torch.empty((ns, 1, round32(cout), round32(cin)), dtype=torch.float32, device=x.device)
        call("u3d_conv_wgrad1", dy.data_ptr(), x.data_ptr(), n, cin, d, h, w_, cout, stride, _ptr(st), _ptr(ga),
             _ptr(be), G, part.data_ptr(), ns, _stream())
        return part, ns
    if brick:
        ns = query("u3d_conv_wgrad_brick_splits", n, cin, d, h, w_, cout, stride)
        part = torch.empty((ns, 27, round32(cout), round32(cin)), dtype=torch.float32, device=x.device)
        call("u3d_conv_wgrad_brick", dy.data_ptr(), x.data_ptr(), n, cin, d, h, w_, cout, stride, _ptr(st), _ptr(ga),
             _ptr(be), G, part.data_ptr(), ns, _stream())
        return part, ns
    ns = query("u3d_conv_wgrad_splits", n, cin, d, h, w_, cout, k, stride)
    part = torch.empty((ns, k ** 3, round32(cout), round32(cin)), dtype=torch.float32, device=x.device)
    call("u3d_conv_wgrad", dt_code(x.dtype), dy.data_ptr(), x.data_ptr(), n, cin, d, h, w_, cout, k, stride, _ptr(st),
         _ptr(ga), _ptr(be), G, part.data_ptr(), ns, _stream())
    return part, ns


# sum each weight gradient's slabs right after the launch that wrote them (round 5, cache-resident) instead of in the
# batched standardisation backward at the end: conv_wgrad then returns (partials, 1)
EAGER_SLAB_SUM = os.environ.get("U3D_EAGER_SLAB_SUM", "0") != "0"
EAGER_SLAB_MIN = int(os.environ.get("U3D_EAGER_SLAB_MIN", "2"))  # fewest slabs summed eagerly


def sum_slabs(part, ns, cout, cin):
    """slab 0 of ``part`` [ns, k^3, cout_p, cin_p] <- the sum over slabs (u3d_wgrad_sum_slabs). Returns (part, 1)."""
    if ns > 1:
        call("u3d_wgrad_sum_slabs", part.data_ptr(), ns, part.shape[1], cout, cin, _stream())
    return part, 1


def use_head(dtype, cin, cout, k, stride):
    """The streaming MFMA head kernel (head.hip) serves GN+ReLU + 1^3 conv with cout <= 32 (precls_conv)."""
    return USE_HEAD and dtype == torch.bfloat16 and k == 1 and stride == 1 and cout <= 32 and cin % 16 == 0 \
        and 16 <= cin <= 64


USE_HEAD = True


def head_fwd(x, wpk, cout, bias, gn):
    """x bf16 [n,d,h,w,cin] -> fp32 logits [n,d,h,w,cout] = conv1(relu(gn(x))) + bias."""
    n, cin = x.shape[0], x.shape[-1]
    v = x.numel() // (n * cin)
    y = torch.empty(tuple(x.shape[:-1]) + (cout,), dtype=torch.float32, device=x.device)
    st, ga, be, G = gn if gn is not None else (None, None, None, 0)
    call("u3d_head_fwd", x.data_ptr(), n, v, cin, wpk.data_ptr(), cout, _ptr(bias), _ptr(st), _ptr(ga), _ptr(be), G,
         y.data_ptr(), _stream())
    return y


def head_bwd(dy, wpk_dgrad, cin, dbias=None):
    """dy fp32 [..., cout] -> (dA bf16 [..., cin], dy bf16 [..., round8(cout)]); the bias gradient is written
    into ``dbias`` (sum over all voxels) when given."""
    cout = dy.shape[-1]
    rows = dy.numel() // cout
    if dy.dtype != torch.float32 or not dy.is_contiguous():
        dy = dy.float().contiguous()
    dA = torch.empty(tuple(dy.shape[:-1]) + (cin,), dtype=torch.bfloat16, device=dy.device)
    dyb = torch.empty(tuple(dy.shape[:-1]) + ((cout + 7) // 8 * 8,), dtype=torch.bfloat16, device=dy.device)
    nb = query("u3d_head_bwd_blocks", rows)
    dbp = torch.empty((nb, cout), dtype=torch.float32, device=dy.device)
    call("u3d_head_bwd", dy.data_ptr(), rows, cout, wpk_dgrad.data_ptr(), cin, dA.data_ptr(), dyb.data_ptr(),
         dbp.data_ptr(), _stream())
    if dbias is not None:
        channel_sum(dbp, out=dbias)
    return dA, dyb


# the partial-label loss hands its gradient to the streaming head unformed (loss.DeferredLossGrad) and the head's
# backward forms it in registers (u3d_head_loss_bwd): no fp32 dlogits tensor
HEAD_LOSS_FUSED = os.environ.get("U3D_HEAD_LOSS_FUSED", "1") != "0"


HEAD_GN_PARTS = os.environ.get("U3D_HEAD_GN_PARTS", "1") == "1"
HEAD_CNT_SLOT = 24  # the GN head backward's arrival counter (zeroed, left zeroed)
HEAD_DBIAS_FUSED = os.environ.get("U3D_HEAD_DBIAS_FUSED", "1") == "1"  # 0: two channel-sum launches (A/B)


def head_gn_parts_ok(lg, x0, cin, gn):
    """u3d_head_loss_bwd_gn applies: the head's GN + ReLU prologue input x0 bf16 with 32 channels, voxels per sample a
    multiple of 32 (its blocks never straddle samples)."""
    if not HEAD_GN_PARTS or gn is None or x0.dtype != torch.bfloat16 or cin != 32 or lg.shape[-1] != 16:
        return False
    n = lg.shape[0]
    return query("u3d_head_loss_bwd_gn_bps", n, lg.numel() // (16 * n), cin) > 0


def head_loss_bwd(lg, lab, weights, sums, grad_out, wpk_dgrad, cin, dbias=None, x0=None, gn=None):
    """head_bwd(partial_loss_bwd(lg, lab, weights, sums, grad_out)) for the softmax + BCE loss over 16 classes in one
    pass (u3d_head_loss_bwd): lg fp32 NDHWC [S, ..., 16], lab fp32 [S, ...]; the same (dA, dy bf16) and bias gradient
    bitwise, without the fp32 dlogits tensor.

    ``x0``, ``gn`` = (stats, gamma, beta, groups) of the head's GroupNorm + ReLU prologue (round 6,
    u3d_head_loss_bwd_gn, when head_gn_parts_ok): the GroupNorm backward's partial sums are taken in the same pass;
    returns (dA, dy, parts) with parts [n, bps, cin, 2] for gn_bwd_parts."""
    C = lg.shape[-1]
    rows = lg.numel() // C
    dA = torch.empty(tuple(lg.shape[:-1]) + (cin,), dtype=torch.bfloat16, device=lg.device)
    dyb = torch.empty(tuple(lg.shape[:-1]) + (C,), dtype=torch.bfloat16, device=lg.device)
    if gn is not None:
        require_device(x0)
        n = lg.shape[0]
        v = rows // n
        assert x0.shape[:-1] == lg.shape[:-1] and x0.shape[-1] == cin and x0.is_contiguous(), "head_loss_bwd: x0 shape"
        bps = query("u3d_head_loss_bwd_gn_bps", n, v, cin)
        assert bps > 0, "head_loss_bwd: GN-partials form does not apply (head_gn_parts_ok)"
        dbp = torch.empty((n * bps, C), dtype=torch.float32, device=lg.device)
        parts = torch.empty((n, bps, cin, 2), dtype=torch.float32, device=lg.device)
        st, ga, be, G = gn
        # the bias gradient summed by the launch's last workgroup (zeroed counter in its own workspace slot)
        fused = dbias is not None and HEAD_DBIAS_FUSED
        call("u3d_head_loss_bwd_gn", lg.data_ptr(), lab.data_ptr(), n, v, C, weights.data_ptr(), sums.data_ptr(),
             grad_out.data_ptr(), wpk_dgrad.data_ptr(), cin, dA.data_ptr(), dyb.data_ptr(), dbp.data_ptr(),
             x0.data_ptr(), st.data_ptr(), ga.data_ptr(), be.data_ptr(), G, parts.data_ptr(),
             _ptr(dbias) if fused else None, _ptr(WS.get(256, lg.device, slot=HEAD_CNT_SLOT)) if fused else None,
             _stream())
        if dbias is not None and not fused:
            channel_sum(dbp, out=dbias)
        return dA, dyb, parts
    nb = query("u3d_head_bwd_blocks", rows)
    dbp = torch.empty((nb, C), dtype=torch.float32, device=lg.device)
    call("u3d_head_loss_bwd", lg.data_ptr(), lab.data_ptr(), rows, C, weights.data_ptr(), sums.data_ptr(),
         grad_out.data_ptr(), wpk_dgrad.data_ptr(), cin, dA.data_ptr(), dyb.data_ptr(), dbp.data_ptr(), _stream())
    if dbias is not None:
        channel_sum(dbp, out=dbias)
    return dA, dyb


STEM_SLOT = 13  # the conv1 kernel's fp32 weight table
STEM_WS_BYTES = 27 * 32 * 4  # = u3d_stem_fwd_ws_bytes() (tests/test_host.py); a constant so A/B runs load older builds


def stem_fwd(x_ncdhw, wpk, cout, stride, dtype):
    require_device(x_ncdhw)
    n, cin, d, h, w_ = x_ncdhw.shape
    od, oh, ow = out_dim(d, 3, stride), out_dim(h, 3, stride), out_dim(w_, 3, stride)
    y = torch.empty((n, od, oh, ow, cout), dtype=dtype, device=x_ncdhw.device)
    ws = WS.get(STEM_WS_BYTES, x_ncdhw.device, slot=STEM_SLOT)
    call("u3d_stem_fwd", dt_code(dtype), x_ncdhw.data_ptr(), n, cin, d, h, w_, wpk.data_ptr(), cout, stride,
         y.data_ptr(), ws.data_ptr(), _stream())
    return y


STEM_STATS = os.environ.get("U3D_STEM_STATS", "1") != "0"  # conv1's GroupNorm(16) statistics from its epilogue


def stem_fwd_stats(x_ncdhw, wpk, cout, stride, dtype):
    """stem_fwd that also returns the output's GroupNorm(16) statistics [n,16,2] when the bf16 conv1 kernel runs with
    its epilogue statistics (u3d_stem1_fwd_stats); otherwise (stem_fwd(...), None)."""
    n, cin, d, h, w_ = x_ncdhw.shape
    if STEM_STATS and dtype == torch.bfloat16 and cin == 1 and cout == 32 and stride == 1 and get_option("STEM1") != 0:
        nws = query("u3d_stem1_stats_ws_floats", n, d, h, w_)
        if nws > 0:
            require_device(x_ncdhw)
            y = torch.empty((n, d, h, w_, cout), dtype=dtype, device=x_ncdhw.device)
            stats = torch.empty((n, 16, 2), dtype=torch.float32, device=x_ncdhw.device)
            sp = WS.get(4 * nws, x_ncdhw.device, slot=STEM_STATS_SLOT)
            ws = WS.get(STEM_WS_BYTES, x_ncdhw.device, slot=STEM_SLOT)
            call("u3d_stem1_fwd_stats", x_ncdhw.data_ptr(), n, d, h, w_, wpk.data_ptr(), y.data_ptr(), ws.data_ptr(),
                 sp.data_ptr(), stats.data_ptr(), _stream())
            return y, stats
    return stem_fwd(x_ncdhw, wpk, cout, stride, dtype), None


STEM_STATS_SLOT = 14


def stem_wgrad(dy, x_ncdhw, stride):
    n, cin, d, h, w_ = x_ncdhw.shape
    cout = dy.shape[-1]
    ns = query("u3d_stem_wgrad_splits2", dt_code(dy.dtype), n, cin, d, h, w_, cout, stride)
    part = torch.empty((ns, 27, round32(cout), round32(cin)), dtype=torch.float32, device=dy.device)
    call("u3d_stem_wgrad", dt_code(dy.dtype), dy.data_ptr(), x_ncdhw.data_ptr(), n, cin, d, h, w_, cout, stride,
         part.data_ptr(), ns, _stream())
    return part, ns


# ------------------------------------------------------------------------------------------ GroupNorm
def _gn_ws(n, c, v, device):
    return WS.get(query("u3d_gn_workspace_bytes", n, c, v), device, slot=1)


def gn_stats(x, groups):
    n, c = x.shape[0], x.shape[-1]
    v = x.numel() // (n * c)
    st = torch.empty((n, groups, 2), dtype=torch.float32, device=x.device)
    call("u3d_gn_stats", dt_code(x.dtype), x.data_ptr(), n, c, v, groups, st.data_ptr(),
         _gn_ws(n, c, v, x.device).data_ptr(), _stream())
    return st


GN_MATERIALIZE_BYTES = 32 << 20
GN_MATERIALIZE_MIN_C = 64


def gn_apply(x, stats, gamma, beta, groups):
    """relu(group_norm(x)) materialised (NDHWC, same dtype)."""
    n, c = x.shape[0], x.shape[-1]
    v = x.numel() // (n * c)
    y = torch.empty_like(x)
    call("u3d_gn_apply", dt_code(x.dtype), x.data_ptr(), n, c, v, groups, stats.data_ptr(), gamma.data_ptr(),
         beta.data_ptr(), y.data_ptr(), _stream())
    return y


def gn_bwd(da, x, stats, gamma, beta, groups, dx=None, accumulate=False, dgamma=None, dbeta=None, acc_params=False):
    n, c = x.shape[0], x.shape[-1]
    v = x.numel() // (n * c)
    if dx is None:
        dx = torch.empty_like(x)
        accumulate = False
    call("u3d_gn_bwd", dt_code(x.dtype), da.data_ptr(), x.data_ptr(), n, c, v, groups, stats.data_ptr(),
         gamma.data_ptr(), beta.data_ptr(), dx.data_ptr(), int(accumulate), _ptr(dgamma), _ptr(dbeta), int(acc_params),
         _gn_ws(n, c, v, x.device).data_ptr(), _stream())
    return dx


def gn_bwd_parts(da, x, parts, stats, gamma, beta, groups, dx=None, accumulate=False, dgamma=None, dbeta=None,
                 acc_params=False):
    """gn_bwd from the per-workgroup partials of conv_dgrad_gn (no partial pass over da and x)."""
    n, c = x.shape[0], x.shape[-1]
    v = x.numel() // (n * c)
    if dx is None:
        dx = torch.empty_like(x)
        accumulate = False
    call("u3d_gn_bwd_parts", da.data_ptr(), x.data_ptr(), n, c, v, groups, stats.data_ptr(), gamma.data_ptr(),
         beta.data_ptr(), parts.data_ptr(), parts.shape[1], dx.data_ptr(), int(accumulate), _ptr(dgamma), _ptr(dbeta),
         int(acc_params), _gn_ws(n, c, v, x.device).data_ptr(), _stream())
    return dx


def gn_bwd2(da1, da2, x, stats, gn1, gn2, groups, dx=None, accumulate=False, dparams1=(None, None),
            dparams2=(None, None), da2_s2=False):
    """Two GroupNorm+ReLU consumers of x (same statistics): gn_k = (gamma_k, beta_k); one fused backward.
    da2_s2: da2 is a stride-2 1^3 conv's data gradient at that conv's output resolution (conv_dgrad_1x1s2_compact)."""
    n, c = x.shape[0], x.shape[-1]
    v = x.numel() // (n * c)
    if dx is None:
        dx = torch.empty_like(x)
        accumulate = False
    if da2_s2:
        d, h, w_ = x.shape[1:4]
        assert tuple(da2.shape) == (n, out_dim(d, 1, 2), out_dim(h, 1, 2), out_dim(w_, 1, 2), c), da2.shape
        call("u3d_gn_bwd2_s2", dt_code(x.dtype), da1.data_ptr(), da2.data_ptr(), x.data_ptr(), n, c, d, h, w_, groups,
             stats.data_ptr(), gn1[0].data_ptr(), gn1[1].data_ptr(), gn2[0].data_ptr(), gn2[1].data_ptr(),
             dx.data_ptr(), int(accumulate), _ptr(dparams1[0]), _ptr(dparams1[1]), _ptr(dparams2[0]),
             _ptr(dparams2[1]), 0, _gn_ws(n, c, v, x.device).data_ptr(), _stream())
        return dx
    call("u3d_gn_bwd2", dt_code(x.dtype), da1.data_ptr(), da2.data_ptr(), x.data_ptr(), n, c, v, groups,
         stats.data_ptr(), gn1[0].data_ptr(), gn1[1].data_ptr(), gn2[0].data_ptr(), gn2[1].data_ptr(), dx.data_ptr(),
         int(accumulate), _ptr(dparams1[0]), _ptr(dparams1[1]), _ptr(dparams2[0]), _ptr(dparams2[1]), 0,
         _gn_ws(n, c, v, x.device).data_ptr(), _stream())
    return dx


GN_BWD_PAIRS = os.environ.get("U3D_GN_PAIRS", "1") != "0"  # fuse gn1 + downsample-GN backward of a block


# ------------------------------------------------------------------------------------------ upsample
def upsample2x_add(x, skip=None):
    n, d, h, w_, c = x.shape
    y = torch.empty((n, 2 * d, 2 * h, 2 * w_, c), dtype=x.dtype, device=x.device)
    call("u3d_upsample2x_add", dt_code(x.dtype), x.data_ptr(), n, c, d, h, w_, _ptr(skip), y.data_ptr(), _stream())
    return y


UP_STATS = os.environ.get("U3D_UP_STATS", "1") != "0"  # decoder upsample + skip: GroupNorm(16) stats in the epilogue


def upsample2x_add_stats(x, skip=None):
    """upsample2x_add that also returns the output's GroupNorm(16) statistics [n,16,2] from its epilogue (bf16,
    u3d_upsample2x_add_stats); otherwise (upsample2x_add(...), None)."""
    n, d, h, w_, c = x.shape
    if UP_STATS and x.dtype == torch.bfloat16 and get_option("UP_QUAD") != 0:
        nws = query("u3d_upsample2x_stats_ws_floats", n, c, d, h, w_)
        if nws > 0:
            y = torch.empty((n, 2 * d, 2 * h, 2 * w_, c), dtype=x.dtype, device=x.device)
            stats = torch.empty((n, 16, 2), dtype=torch.float32, device=x.device)
            sp = WS.get(4 * nws, x.device, slot=UP_STATS_SLOT)
            call("u3d_upsample2x_add_stats", x.data_ptr(), n, c, d, h, w_, _ptr(skip), y.data_ptr(), sp.data_ptr(),
                 stats.data_ptr(), _stream())
            return y, stats
    return upsample2x_add(x, skip), None


UP_STATS_SLOT = 15


def upsample2x_bwd(dy, in_shape, dx=None, accumulate=False):
    n, d, h, w_, c = in_shape
    if dx is None:
        dx = torch.empty(in_shape, dtype=dy.dtype, device=dy.device)
        accumulate = False
    call("u3d_upsample2x_bwd", dt_code(dy.dtype), dy.data_ptr(), n, c, d, h, w_, dx.data_ptr(), int(accumulate),
         _stream())
    return dx


# ------------------------------------------------------------------------------------------ misc
def add_(y, x):
    call("u3d_add_inplace", dt_code(y.dtype), y.data_ptr(), x.data_ptr(), y.numel(), _stream())
    return y


def cast(x, dtype, pad_to=1):
    """Convert dtype and zero-pad the channel (last) dim to a multiple of ``pad_to``."""
    c = x.shape[-1]
    cp = (c + pad_to - 1) // pad_to * pad_to
    if x.dtype == dtype and cp == c:
        return x
    y = torch.empty(tuple(x.shape[:-1]) + (cp,), dtype=dtype, device=x.device)
    call("u3d_cast", dt_code(x.dtype), x.data_ptr(), dt_code(dtype), y.data_ptr(), x.numel() // c, c, cp, _stream())
    return y


def channel_sum(x, out=None, accumulate=False):
    c = x.shape[-1]
    rows = x.numel() // c
    if out is None:
        out = torch.empty((c,), dtype=torch.float32, device=x.device)
        accumulate = False
    ws = WS.get(query("u3d_channel_sum_workspace_bytes", rows, c), x.device, slot=2)
    call("u3d_channel_sum", dt_code(x.dtype), x.data_ptr(), rows, c, out.data_ptr(), int(accumulate), ws.data_ptr(),
         _stream())
    return out


# ------------------------------------------------------------------------------------------ loss / metric
def partial_target(labels, mask, lmin=1, lmax=13):
    """labels fp32 (any shape, leading dim S) with organs the mask marks unlabelled set to 0 (A12)."""
    require_device(labels)
    lab = labels.float().contiguous()
    m = torch.as_tensor(mask).to(device=labels.device, dtype=torch.int64)
    S = lab.shape[0]
    V = lab.numel() // S
    if m.dim() == 1:
        stride, M = 0, m.numel()
    else:
        assert m.shape[0] == S, "one mask row per sample"
        stride, M = m.shape[1], m.shape[1]
    m = m.contiguous()
    out = torch.empty_like(lab)
    call("u3d_partial_target", lab.data_ptr(), S, V, m.data_ptr(), stride, M, lmin, lmax, out.data_ptr(), _stream())
    return out


def partial_loss_fwd(logits, labels, weights, softmax=True, uce=True):
    """logits fp32 [S, ..., C] NDHWC-contiguous, labels fp32 [S, ...] -> (loss fp32[1], sums fp64[C,4])."""
    S, C = logits.shape[0], logits.shape[-1]
    V = logits.numel() // (S * C)
    sums = torch.empty((C, 4), dtype=torch.float64, device=logits.device)
    loss = torch.empty((1,), dtype=torch.float32, device=logits.device)
    ws = WS.get(query("u3d_loss_workspace_bytes", S, V, C), logits.device, slot=3)
    call("u3d_partial_loss_fwd", logits.data_ptr(), labels.data_ptr(), S, V, C, int(softmax), weights.data_ptr(),
         int(uce), sums.data_ptr(), loss.data_ptr(), ws.data_ptr(), _stream())
    return loss, sums


def partial_loss_bwd(logits, labels, weights, sums, grad_out, softmax=True, uce=True, out_dtype=torch.float32):
    S, C = logits.shape[0], logits.shape[-1]
    V = logits.numel() // (S * C)
    dl = torch.empty(logits.shape, dtype=out_dtype, device=logits.device)
    call("u3d_partial_loss_bwd", dt_code(out_dtype), logits.data_ptr(), labels.data_ptr(), S, V, C, int(softmax),
         weights.data_ptr(), int(uce), sums.data_ptr(), grad_out.data_ptr(), dl.data_ptr(), _stream())
    return dl


def dice_metric(logits, labels, num_class, want_argmax=False):
    """logits fp32 NDHWC [S, ..., C]; returns (metrics [num_class, 3] = dice/sens/prec, counts, argmax|None)."""
    S, C = logits.shape[0], logits.shape[-1]
    V = logits.numel() // (S * C)
    counts = torch.empty((S, num_class, 3), dtype=torch.int64, device=logits.device)
    metrics = torch.empty((num_class, 3), dtype=torch.float32, device=logits.device)
    am = torch.empty(logits.shape[:-1], dtype=torch.int64, device=logits.device) if want_argmax else None
    call("u3d_dice_metric", logits.data_ptr(), labels.data_ptr(), S, V, C, num_class, counts.data_ptr(),
         metrics.data_ptr(), _ptr(am), _stream())
    return metrics, counts, am
