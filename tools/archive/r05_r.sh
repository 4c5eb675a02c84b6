#!/bin/bash
# Round 5 batch r: the small-volume conv's tail (slab stores, counters, combine, finalize) at 12^3 / 6^3, forward and
# data gradient.
TAG=${1:-r05_r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for c in small12 small06 smalldg12 smalldg06; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c > $O/stamps_$c.log 2>&1 || { cat $O/stamps_$c.log; exit 1; }
  echo "== $c"; grep -v "amdgpu.ids\|wave [1-7]:" $O/stamps_$c.log
done
