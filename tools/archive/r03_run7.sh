#!/bin/bash
# r03: cap on the weight-gradient split-K slab bytes per launch (U3D_WG_SLAB_KB): step A/B and deep-level kernels
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03p
mkdir -p $O
cd $R
for cap in 0 8192 2048; do
  echo "cap=$cap" >> $O/k.log
  U3D_WG_SLAB_KB=$cap timeout -k 10 200 python tools/kbench.py wgrad12 wgrad6 wgrad24 2>&1 | grep -v amdgpu.ids >> $O/k.log || exit 1
done
cat $O/k.log
bash tools/ab.sh r03p/ab1 "U3D_WG_SLAB_KB=0" "U3D_WG_SLAB_KB=8192" 3 || exit 1
bash tools/ab.sh r03p/ab2 "U3D_WG_SLAB_KB=0" "U3D_WG_SLAB_KB=2048" 3 || exit 1
