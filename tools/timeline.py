"""Per-step timeline of a rocprofv3 kernel trace (graph-replayed bench): wall time, union busy time (any
stream), per-stream busy, and the idle gaps. Usage: python tools/timeline.py TRACE_DIR [marker-substring]"""
import csv
import sys

d = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "stem1_"
rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows]
starts = [k[0] for k in ks if marker in k[3]]
print(f"{len(starts)} steps (marker {marker})")
tot = {}
for i in range(len(starts) - 1):
    a, b = starts[i], starts[i + 1]
    seg = [k for k in ks if a <= k[0] < b]
    wall = (b - a) / 1e3
    # union of busy intervals
    iv = sorted((s, min(e, b)) for s, e, _, _ in seg)
    busy, cs, ce = 0, None, None
    gaps = []
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
                gaps.append((s - ce, s))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    per = {}
    for s, e, st, _ in seg:
        per[st] = per.get(st, 0) + (e - s)
    big = sorted(gaps, reverse=True)[:3]
    print(f"step {i}: wall {wall:7.3f} ms  union-busy {busy / 1e3:7.3f}  idle {wall - busy / 1e3:6.3f}  "
          f"streams " + " ".join(f"{k}:{v / 1e6:.3f}" for k, v in sorted(per.items())) +
          f"  largest gaps(us) {[round(g / 1e3, 1) for g, _ in big]}")

# per-kernel totals over the replayed steps (skipping the first two markers: eager warm-up / capture)
if len(starts) > 4:
    a, b = starts[2], starts[-1]
    nst = len(starts) - 3
    agg = {}
    for s, e, _, nm in ks:
        if a <= s < b:
            key = nm.split("(")[0].replace("void ", "")[:70]
            c, t = agg.get(key, (0, 0))
            agg[key] = (c + 1, t + e - s)
    tot = sum(t for _, t in agg.values())
    print(f"--- kernels over {nst} steps: {tot / nst / 1e3:.1f} us/step")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{t / nst / 1e3:8.1f} us/step {100 * t / tot:5.1f}%  n/step={c / nst:4.1f}  {k}")
