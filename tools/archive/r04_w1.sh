#!/bin/bash
# r04: 1^3 weight gradient with two 64 KB-LDS workgroups per CU and twice the splits (w1occ2.so) vs one (in-tree)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_w1
mkdir -p $O
cd $R
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "" "$L/w1occ2.so"; do
    echo "== ${v:-in-tree}" >> $O/kab.log
    U3D_LIB=$v timeout -k 10 120 python tools/kbench.py wgrad1_96 wgrad1_s2_96 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
