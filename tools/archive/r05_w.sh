#!/bin/bash
# Round 5 batch w: the small-volume conv's split count at 6^3 / 12^3 (U3D_SMALL_WGS: workgroups aimed at), the step's
# forms (statistics / GroupNorm-backward finalize in the launch).
TAG=${1:-r05_w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for w in 256 128 64 32 256; do
  U3D_SMALL_WGS=$w timeout -k 10 120 python tools/kbench.py fwd6st dgrad6gb fwd12st dgrad12gb > $O/kb.log 2>&1 || { cat $O/kb.log; exit 1; }
  echo "== SMALL_WGS $w"; grep -v amdgpu.ids $O/kb.log
done
