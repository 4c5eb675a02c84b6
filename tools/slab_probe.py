"""Print the weight-gradient slab reductions of one bench step: per weight (shape, nsplit, MB read by the slab sum)."""
import os
import sys

sys.argv = ["bench.py", "--no-cpu", "--no-roofline", "--steps", "1", "--warmup", "0"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-pl_amd"))
from u3d import ops  # noqa: E402

_orig = ops.wstd_bwd_batch
seen = []


def probe(items):
    for part, ns, w, *_ in items:
        seen.append((tuple(w.shape), ns, part.numel() * 4 / 1e6 if ns > 1 else 0.0))
    return _orig(items)


ops.wstd_bwd_batch = probe
import bench  # noqa: E402

bench.main()
tot = 0.0
for shp, ns, mb in seen[:len(seen)]:
    print(f"{str(shp):24s} ns={ns:4d} slabMB={mb:8.1f}")
    tot += mb
print(f"calls={len(seen)} total slab MB={tot:.1f}")
