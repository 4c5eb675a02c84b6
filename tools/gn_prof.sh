#!/bin/bash
# GroupNorm kernels at every trunk level (graph-replayed, HIP events): tools/gn_prof.sh TAG
TAG=${1:-gn}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
cases=""
for k in stats apply bwd bwd2; do for l in 96 48 24 12 6; do cases="$cases gn$k$l"; done; done
timeout -k 10 200 python tools/kbench.py $cases 2>&1 | grep -v amdgpu.ids | tee $O/gn.txt
