#!/bin/bash
# r04: loss forward block count (U3D_LOSS_NB build variants; 161 VGPRs = 3 waves per SIMD = 768 resident blocks)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_u
mkdir -p $O
cd $R
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "$L/lnb256.so" "$L/lnb384.so" "$L/lnb512.so"; do
    echo "== ${v:-in-tree 1024}" >> $O/kab.log
    U3D_LIB=$v timeout -k 10 120 python tools/kbench.py loss96 lossb96 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
