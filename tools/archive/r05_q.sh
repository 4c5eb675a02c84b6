#!/bin/bash
# Round 5 batch q: where the small-volume conv's time goes (stamps at 12^3 / 6^3), kernel times.
TAG=${1:-r05_q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for c in small12 small06; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c > $O/stamps_$c.log 2>&1; echo "== $c"; grep -v amdgpu.ids $O/stamps_$c.log | head -12
done
timeout -k 10 120 python tools/kbench.py fwd12 dgrad12 fwd6 dgrad6 > $O/kb.log 2>&1; grep -v amdgpu.ids $O/kb.log
