"""In-kernel stamps of a -DU3D_STAMPS build (tools/build_variant.sh libu3d_stamps -DU3D_STAMPS; run with
U3D_LIB=.../libu3d_stamps.so): the clock the chip holds inside the weight-gradient ring at 2x96^3 (s_memtime over
s_memrealtime x 100 MHz, median over workgroups, after >= 2 s of back-to-back launches on random data,
MI355X_MICROARCH.md DVFS item 6) and where its waves spend their cycles (staged-load wait + LDS writes, MFMA compute,
barrier). Usage: python tools/stamps.py [wgrad96|wgrad48|...] [seconds]"""
import ctypes
import os
import statistics
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from u3d import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
case = sys.argv[1] if len(sys.argv) > 1 else "wgrad96"
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 2.5
ring = not case.startswith("wgrad")
s2 = case.startswith("s2ring")
small = case.startswith("small")
smalldg = case.startswith("smalldg")
s, c = {"96": (96, 32), "48": (48, 64), "24": (24, 128), "12": (12, 256), "06": (6, 256)}[case[-2:]]
x = torch.randn((2, s, s, s, c), device=dev).to(torch.bfloat16)
dy = torch.randn_like(x)
gn = (ops.gn_stats(x, 16), torch.ones(c, device=dev), torch.zeros(c, device=dev), 16)
w = torch.randn(c, c, 3, 3, 3, device=dev)
pf, pd, _ = ops.wstd_fwd(w, torch.bfloat16, True)
fn = {"wgrad": lambda: ops.conv_wgrad(dy, x, 3, 1, gn, brick="ring"),
      "fwd": lambda: ops.conv_fwd_stats(x, pf, c, 3, 1, gn, residual=x),
      "fwdnores": lambda: ops.conv_fwd_stats(x, pf, c, 3, 1, gn),
      "dgradgn": lambda: ops.conv_dgrad_gn(dy, pd, c, x, 3, 1, gn),
      "dgrad": lambda: ops.conv_dgrad(dy, pd, c, x.shape[:4], 3, 1)}.get(case[:-2])
if small:  # the small-volume conv (conv_small.hip) at 12^3 / 6^3, 256 -> 256 with the GN prologue
    c = 256
    x = torch.randn((2, s, s, s, c), device=dev).to(torch.bfloat16)
    gn = (ops.gn_stats(x, 16), torch.ones(c, device=dev), torch.zeros(c, device=dev), 16)
    w3 = torch.randn(c, c, 3, 3, 3, device=dev)
    pf3, _, _ = ops.wstd_fwd(w3, torch.bfloat16, True, need_dgrad=False)
    fn = lambda: ops.conv_fwd_stats(x, pf3, c, 3, 1, gn)  # noqa: E731 (the step's form: output statistics in the combine)
    if smalldg:  # the data gradient with the GroupNorm-backward partials + finalize in its combine
        _, pd3, _ = ops.wstd_fwd(w3, torch.bfloat16, True)
        dy = torch.randn_like(x)
        dgam, dbet = torch.empty(c, device=dev), torch.empty(c, device=dev)
        fn = lambda: ops.conv_dgrad_gn(dy, pd3, c, x, 3, 1, gn, dgb=lambda: (dgam, dbet))  # noqa: E731
if s2:  # the stride-2 forward ring (conv_s2.hip): 32 -> 64
    w2 = torch.randn(64, 32, 3, 3, 3, device=dev)
    pf2, _, _ = ops.wstd_fwd(w2, torch.bfloat16, True, need_dgrad=False)
    fn = lambda: ops.conv_fwd_stats(x, pf2, 64, 3, 2, gn)  # noqa: E731
fn()
torch.cuda.synchronize()
t0 = time.time()
n = 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
while time.time() - t0 < secs:
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    n += 20
us = e0.elapsed_time(e1) / 20 * 1e3
buf = np.zeros(4096 * 8 * 8, dtype=np.uint64)
h = _lib.lib()
if small:
    assert h.u3d_diag_small_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes)) == 0
    nwg = 1024
    names = ("chunk MFMAs", "commit+barrier", "barrier")
elif s2:
    assert h.u3d_diag_s2_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes)) == 0
    nwg = 256
    names = ("write+load-wait", "compute", "barrier")
elif ring:
    assert h.u3d_diag_ring_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes)) == 0
    nwg = 256
    names = ("steps", "step heads", "barrier")
else:
    assert h.u3d_diag_wgrad_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(buf.nbytes)) == 0
    nwg = _lib.query("u3d_conv_wgrad_ring_splits", 2, c, s, s, s, c) * (ops.round32(c) // 32) ** 2
    names = ("write+load-wait", "compute", "barrier")
b = buf.reshape(4096, 8, 8)[:nwg].astype(np.float64)
b = b[(b[:, :, 1] - b[:, :, 0]).min(axis=1) > 0]  # workgroups that ran (the grid may be smaller than nwg)
nwg = len(b)
clk = (b[:, 0, 1] - b[:, 0, 0]) / np.maximum(1, b[:, 0, 3] - b[:, 0, 2]) * 100.0  # MHz
wall = b[:, :, 1] - b[:, :, 0]
print(f"{case}: {n} launches, last 20 avg {us:.1f} us/launch, workgroups {nwg}")
print(f"  in-kernel clock: median {np.median(clk):.0f} MHz (p10 {np.percentile(clk, 10):.0f}, p90 {np.percentile(clk, 90):.0f})")
print(f"  workgroup span: median {np.median(wall[:, 0]) / np.median(clk):.1f} us, max {wall[:, 0].max() / np.median(clk):.1f} us")
r0, r1 = b[:, 0, 2], b[:, 0, 3]  # s_memrealtime (100 MHz) at the workgroup's first / last stamp
print(f"  starts spread over {(r0.max() - r0.min()) / 100:.1f} us (p90 {(np.percentile(r0, 90) - r0.min()) / 100:.1f}), "
      f"ends over {(r1.max() - r1.min()) / 100:.1f} us; first start to last end {(r1.max() - r0.min()) / 100:.1f} us")
steps = b[:, :, 7].astype(np.uint64)
for w in range(8):
    tot = wall[:, w]
    fr = [b[:, w, k] / tot for k in (4, 5, 6)]
    print(f"  wave {w}: " + "  ".join(f"{nm} {np.median(f):.3f}" for nm, f in zip(names, fr)) +
          f"  other {1 - np.median(fr[0] + fr[1] + fr[2]):.3f}  steps {int(np.median(steps[:, w] & np.uint64(0xffffffff)))}"
          f" compute-steps {int(np.median(steps[:, w] >> np.uint64(32)))}")
if small:  # the tail after the main loop (TailStamps: slab stores, their drain, the tile counter, the combine, ...)
    tb = np.zeros(256 * 64, dtype=np.uint64)
    assert h.u3d_diag_small_tail(ctypes.c_void_p(tb.ctypes.data), ctypes.c_longlong(tb.nbytes)) == 0
    t = tb.reshape(1024, 16)[:nwg].astype(np.float64)
    mhz = np.median(clk)
    segs = ("slab stores issued", "stores drained", "tile counter", "combine", "partials stored", "stats counter",
            "finalize")
    for lab, sel in (("all", t[:, 3] > 0), ("tile-last", t[:, 4] > 0), ("final", t[:, 7] > 0)):
        q = t[sel]
        if not len(q):
            continue
        row = []
        for k, nm in enumerate(segs, start=1):
            ok = (q[:, k] > 0) & (q[:, k - 1] > 0)
            if ok.any():
                row.append(f"{nm} {np.median(q[ok, k] - q[ok, k - 1]) / mhz:.2f}")
        print(f"  tail ({lab}, {len(q)} wgs, us): " + "  ".join(row))
    rend = t[:, 8]
    print(f"  first start to last exit {(rend.max() - r0.min()) / 100:.1f} us; main-loop ends to exits: median "
          f"{np.median(rend - r1) / 100:.1f} us, max {(rend - r1).max() / 100:.1f} us")
