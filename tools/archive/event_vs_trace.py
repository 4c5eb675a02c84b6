"""Event-vs-trace experiment for the dominant kernel: the production ring conv launch (GN prologue +
residual + statistics) at 2x96^3, each launch bracketed by its own HIP events, in two regimes:
  idle  — the host sleeps 200 us before each launch (the queue is empty when the dispatch arrives, as inside the
          eager training step, where host-side gaps of ~5 us precede most launches);
  busy  — a 1 ms filler kernel (torch matmul) is queued first, so the dispatch waits in a non-empty queue.
Run under rocprofv3 --kernel-trace; prints one JSON line with the per-regime event averages (the trace side is
read afterwards by matching the launch order). Usage: python tools/event_vs_trace.py"""
import json
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multimodal-pl_amd")]
import torch  # noqa: E402
from u3d import ops  # noqa: E402

dev = torch.device("cuda:0")
x = torch.randn((2, 96, 96, 96, 32), device=dev).to(torch.bfloat16)
w = torch.randn(32, 32, 3, 3, 3, device=dev)
pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
st = ops.gn_stats(x, 16)
ga, be = torch.ones(32, device=dev), torch.zeros(32, device=dev)
a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    ops.conv_fwd_stats(x, pf, 32, 3, 1, (st, ga, be, 16), residual=x)
torch.cuda.synchronize()
res = {}
for regime in ("idle", "busy", "idle", "busy"):
    ops.PROBE = probes = []
    for _ in range(10):
        if regime == "idle":
            torch.cuda.synchronize()
            time.sleep(2e-4)
        else:
            for _ in range(8):
                a @ a
        ops.conv_fwd_stats(x, pf, 32, 3, 1, (st, ga, be, 16), residual=x)
    torch.cuda.synchronize()
    ops.PROBE = None
    d = [e0.elapsed_time(e1) * 1e3 for e0, e1, _ in probes]
    res.setdefault(regime, []).extend(d)
print(json.dumps({k: round(sum(v) / len(v), 1) for k, v in res.items()} | {"order": "idle,busy,idle,busy x10"}))
