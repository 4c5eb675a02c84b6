"""Steady-state steps of a rocprofv3 kernel trace of bench.py (the summaries count only the timed
graph replays, not the eager / capture warm-ups, whose first step spans 1.6 s and whose clock ramps).

A step starts at the launch of the stem kernel (the first libu3d kernel of every 2x96^3 step: conv1 on the input volume);
`steady(rows, k)` returns the dispatch rows of the LAST k steps (a step ends where the next one starts) and the
per-step wall times."""
import re

MARKER = r"u3d::stem1_(fwd|mfma)_kernel"


def _t(r, key):
    return int(r[key])


def steady(rows, k, marker=MARKER):
    """The last k steps: the final one runs from the last marker to the end of the trace (bench.py launches nothing on
    the GPU after its timed steps when run with --no-roofline --no-infer --no-mixed --no-cpu)."""
    rows = sorted(rows, key=lambda r: _t(r, "Start_Timestamp"))
    starts = [i for i, r in enumerate(rows) if re.search(marker, r["Kernel_Name"])]
    if not starts:
        raise SystemExit(f"trace_steps: no '{marker}' launch in the trace")
    k = min(k, len(starts))
    sel = starts[-k:] + [len(rows)]
    out, walls = [], []
    for a, b in zip(sel[:-1], sel[1:]):
        out.extend(rows[a:b])
        end = _t(rows[b], "Start_Timestamp") if b < len(rows) else max(_t(r, "End_Timestamp") for r in rows[a:b])
        walls.append((end - _t(rows[a], "Start_Timestamp")) / 1e3)
    return out, walls, k
