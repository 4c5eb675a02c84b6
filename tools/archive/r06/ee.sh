#!/bin/bash
# round 6: GroupNorm reduction grid per kernel kind (kbench at 96^3 / 48^3): which GN kernels gain from more blocks
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06ee; mkdir -p $O; cd $R
for r in 1 2; do for b in 128 192 256; do echo "== GN_MAXBLK=$b" >> $O/kb.log; U3D_GN_MAXBLK=$b timeout -k 10 150 python tools/kbench.py gnbwd2s96 gnbwd96 gnstats96 gnbwd2s48 gnbwd2s24 gnbwd48 >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
