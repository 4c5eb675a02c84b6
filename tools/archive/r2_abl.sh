#!/bin/bash
# Timing ablations of the ring v2 plain forward (wrong results by design; kbench only)
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for a in 0 1 2 4 8 12 14 15 16 32 46; do
  echo "== ABL $a"
  U3D_R2_ABL=$a timeout -k 10 60 python tools/kbench.py fwd96_plain 2>&1 | grep -v amdgpu.ids | tee -a $O/kbench.log || exit 1
done
