#!/bin/bash
# conv_small split-K target (U3D_SMALL_WGS 256 / 512 / 1024): micro-benchmarks and step A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_swgs
mkdir -p $O
cd $R
for t in 256 512 768 1024; do U3D_SMALL_WGS=$t timeout -k 10 120 python tools/kbench.py fwd12 dgrad12 fwd6nogn 2>/dev/null | sed "s/^/wgs=$t /"; done | tee $O/kbench.log
bash tools/ab.sh r02s3_swgs/ab "U3D_SMALL_WGS=512" "U3D_SMALL_WGS=1024" 2 || exit 1
bash tools/ab.sh r02s3_swgs/ab2 "U3D_SMALL_WGS=512" "U3D_SMALL_WGS=256" 2 || exit 1
