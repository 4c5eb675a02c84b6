#!/bin/bash
# r04: GroupNorm reduction block cap (U3D_GN_MAXBLK) per GN kernel family at 2 x 96^3 (kbench, graph replay)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_t
mkdir -p $O
cd $R
for i in 1 2; do
  for v in 256 512 1024; do
    echo "== GN_MAXBLK=$v" >> $O/kab.log
    U3D_GN_MAXBLK=$v timeout -k 10 120 python tools/kbench.py gnbwd2s96 gnbwd96 gnstats96 gnbwd2s48 gnbwd48 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
