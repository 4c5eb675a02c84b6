#!/bin/bash
# r04: voxels per load round in the GN statistics / backward-partial passes: 8 / 4 (in-tree) vs 16 / 8 and 4 / 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_z
mkdir -p $O
cd $R
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "" "$L/gnr16.so" "$L/gnr4.so"; do
    echo "== ${v:-in-tree}" >> $O/kab.log
    U3D_LIB=$v timeout -k 10 120 python tools/kbench.py gnstats96 gnstats48 gnstats12 gnbwd96 gnbwd48 gnbwd12 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
