#!/bin/bash
# Round 5 batch k: workgroup spans vs kernel time of the 96^3 rings and the stride-2 ring (stamps build).
TAG=${1:-r05_k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for c in fwd96 fwdnores96 dgradgn96 wgrad96 wgrad48 s2ring96; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c > $O/stamps_$c.log 2>&1; echo "== $c"; grep -v amdgpu.ids $O/stamps_$c.log | head -5
done
timeout -k 10 120 python tools/kbench.py fwd96 fwd96_nores dgrad96gn wgrad96 wgrad48 fwds2ring > $O/kb.log 2>&1; grep -v amdgpu.ids $O/kb.log
