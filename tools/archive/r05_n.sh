#!/bin/bash
# Round 5 batch n: fixed launch cost of the ring kernels; ring stamps from kernel entry.
TAG=${1:-r05_n}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 120 python tools/r05_tiny.py > $O/tiny.log 2>&1; grep -v amdgpu.ids $O/tiny.log
for c in fwdnores96 dgradgn96; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c > $O/stamps_$c.log 2>&1; echo "== $c"; grep -v amdgpu.ids $O/stamps_$c.log | sed -n '1,6p;10p'
done
