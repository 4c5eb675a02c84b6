"""Timing ablations of the 96^3 ring conv (diagnostic build, tools/build_variant.sh libu3d_diag -DU3D_RING_EXP):
U3D_LIB=multimodal-pl_amd/u3d/libu3d_diag.so python tools/ring_ablate.py [exp ...]. Results of the ablated launches
are wrong by design; only their time is read. Each case is timed twice per variant, interleaved with the baseline."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
import kbench  # noqa: E402
from u3d import ops  # noqa: E402

exps = [int(a) for a in sys.argv[1:]] or [0, 1, 2, 4, 8, 16, 32, 3, 12, 18]
cases = ["fwd96", "fwd96_nores", "dgrad96"]
for rep in range(2):
    for e in exps:
        with ops.option("RING_EXP", e):
            row = []
            for c in cases:
                us, flop = kbench.CASES[c]()
                row.append(f"{c} {us:7.1f} us")
        print(f"exp {e:3d}: " + "  ".join(row), flush=True)
