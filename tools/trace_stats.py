"""Kernels per step and GroupNorm kernel time per step from a rocprofv3 kernel trace (run_kernel_trace.csv):
python tools/trace_stats.py DIR [steps]. GroupNorm kernels: names with gn_ / _gn_finalize / gn16 (the separate passes and
finalize launches; the statistics and partials fused into conv epilogues are counted with their conv)."""
import collections
import csv
import re
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
if len(sys.argv) > 3 and sys.argv[3] == "steady":  # only the last `steps` complete (timed) steps
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import trace_steps
    rows, _, steps = trace_steps.steady(rows, steps)
gn = collections.defaultdict(float)
n_u3d = 0
for r in rows:
    nm = r["Kernel_Name"]
    dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "u3d::" in nm:
        n_u3d += 1
    if re.search(r"u3d::(gn_|ring_gn_finalize|pbrick_gn_finalize|gn_bwd)", nm):
        gn[re.sub(r"\(.*", "", nm)] += dt
print(f"kernels per step: {len(rows) / steps:.1f} (u3d {n_u3d / steps:.1f})")
print(f"GroupNorm kernels per step: {sum(gn.values()) / steps / 1e3:.3f} ms")
for k, v in sorted(gn.items(), key=lambda kv: -kv[1]):
    print(f"  {v / steps:8.1f} us  {k}")
