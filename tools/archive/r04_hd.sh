#!/bin/bash
# r04: head forward / backward grid cap (U3D_HEAD_NB: 2048 in-tree vs 768 / 1024 / 1280 build variants)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_hd
mkdir -p $O
cd $R
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "" "$L/hnb768.so" "$L/hnb1024.so" "$L/hnb1280.so"; do
    echo "== ${v:-in-tree}" >> $O/kab.log
    U3D_LIB=$v timeout -k 10 120 python tools/kbench.py headf96 headb96 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
