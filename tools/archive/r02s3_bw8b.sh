#!/bin/bash
# 8-wide bricks at 48^3 too? micro-benchmarks with U3D_CONVG_BW8 forced on / off, step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_bw8b
mkdir -p $O
cd $R
for b in 1 0; do U3D_CONVG_BW8=$b timeout -k 10 120 python tools/kbench.py fwd48 dgrad48 2>/dev/null | sed "s/^/bw8=$b /"; done | tee $O/kbench.log
