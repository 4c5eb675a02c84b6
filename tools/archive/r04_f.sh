#!/bin/bash
# r04: implicit-GEMM register pipeline depth (K-steps of loads in flight) for the stride-2 forward convs: in-tree
# (D = 3 / 2 for 32- / 64-channel K-steps) vs libu3d_d4 (4 / 3) vs libu3d_d6 (6 / 4), kbench, alternating x2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_f
mkdir -p $O
cd $R
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_d4.so" "U3D_LIB=$L/libu3d_d6.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py fwd_s2_96 fwd_s2_48 fwd_s2_24 fwd12nogn fwd6nogn >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
