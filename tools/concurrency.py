"""Persistent ring kernels under a concurrent kernel: the 2x96^3 32->32 ring conv (forward with
the GN prologue + residual + epilogue statistics, and the data gradient) timed alone and while a side-stream kernel
holds K CUs (u3d_diag_occupy: the one-GPU stand-in for RCCL's all-reduce kernels during the data-parallel backward),
static schedule (one fixed plane range per workgroup) vs work queue. Prints one JSON object.
Usage: python tools/concurrency.py [K ...]"""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
import torch  # noqa: E402
from u3d import ops  # noqa: E402
from u3d._lib import call  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    ks = [int(a) for a in sys.argv[1:]] or [8, 32]
    torch.manual_seed(0)
    n, s = 2, 96
    x = (torch.randn((n, s, s, s, 32), device=dev) * 0.5).to(bf)
    r = (torch.randn((n, s, s, s, 32), device=dev) * 0.5).to(bf)
    w = torch.randn(32, 32, 3, 3, 3, device=dev)
    pf, pd, _ = ops.wstd_fwd(w, bf, True)
    gn = (ops.gn_stats(x, 16), torch.ones(32, device=dev), torch.zeros(32, device=dev), 16)
    out = torch.zeros(4, device=dev)
    side = torch.cuda.Stream(device=dev)
    cases = {"fwd": lambda: ops.conv_fwd_stats(x, pf, 32, 3, 1, gn, r),
             "dgrad": lambda: ops.conv_dgrad(x, pd, 32, (n, s, s, s), 3, 1)}
    # the persistent brick data gradients at 48^3 x 64 and 24^3 x 128 (round 3: u3d_convg_brick_q)
    for s2, c2 in ((48, 64), (24, 128)):
        x2 = (torch.randn((n, s2, s2, s2, c2), device=dev) * 0.5).to(bf)
        _, pd2, _ = ops.wstd_fwd(torch.randn(c2, c2, 3, 3, 3, device=dev), bf, True)
        cases[f"dgrad{s2}"] = (lambda x2=x2, pd2=pd2, s2=s2, c2=c2: ops.conv_dgrad(x2, pd2, c2, (n, s2, s2, s2), 3, 1))
    # conv_small data gradient at 12^3 x 256, the stride-2 data gradients 96^3 -> 48^3 and 48^3 -> 24^3, and the
    # stride-1 weight-gradient rings at 96^3 and 48^3 (queue mode: short ranges, u3d.ops.WGRAD_QUEUE)
    x12 = (torch.randn((n, 12, 12, 12, 256), device=dev) * 0.5).to(bf)
    _, pd12, _ = ops.wstd_fwd(torch.randn(256, 256, 3, 3, 3, device=dev), bf, True)
    cases["dgrad12"] = lambda: ops.conv_dgrad(x12, pd12, 256, (n, 12, 12, 12), 3, 1)
    for s3, ci, co in ((96, 32, 64), (48, 64, 128)):
        dy3 = (torch.randn((n, s3 // 2, s3 // 2, s3 // 2, co), device=dev) * 0.5).to(bf)
        _, pd3, _ = ops.wstd_fwd(torch.randn(co, ci, 3, 3, 3, device=dev), bf, True)
        cases[f"dgrad_s2_{s3}"] = (lambda dy3=dy3, pd3=pd3, ci=ci, s3=s3: ops.conv_dgrad(dy3, pd3, ci, (n, s3, s3, s3), 3, 2))
    dyw = (torch.randn((n, s, s, s, 32), device=dev) * 0.5).to(bf)
    cases["wgrad96"] = lambda: ops.conv_wgrad(dyw, x, 3, 1, gn)
    x48 = (torch.randn((n, 48, 48, 48, 64), device=dev) * 0.5).to(bf)
    cases["wgrad48"] = lambda: ops.conv_wgrad(x48, x48, 3, 1, None)

    def timed(fn, reps=10):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = ev(), ev()
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e3

    # occupy-kernel calibration: iterations for ~400 us (covers one ring launch after it)
    it = 200000
    t_occ = timed(lambda: call("u3d_diag_occupy", 8, it, out.data_ptr(), torch.cuda.current_stream().cuda_stream))
    iters = int(it * 400.0 / t_occ)

    def with_hog(fn, k, reps=10):
        ts = []
        for _ in range(reps + 2):
            torch.cuda.synchronize()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                call("u3d_diag_occupy", k, iters, out.data_ptr(), side.cuda_stream)
            a, b = ev(), ev()
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        ts = sorted(ts[2:])
        return ts[len(ts) // 2]

    res = {"occupy_us_per_8wg_200k": round(t_occ, 1), "occupy_iters": iters, "cases": {}}
    for name, fn in cases.items():
        for mode in ("static", "queue"):
            ops.RING_QUEUE = ops.WGRAD_QUEUE = mode == "queue"
            row = {"alone_us": round(timed(fn), 1)}
            for k in ks:
                row[f"with_{k}_cus_held_us"] = round(with_hog(fn, k), 1)
            res["cases"][f"{name}_{mode}"] = row
            print(name, mode, row, file=sys.stderr, flush=True)
    ops.RING_QUEUE = ops.WGRAD_QUEUE = False
    print(json.dumps(res))


if __name__ == "__main__":
    main()
