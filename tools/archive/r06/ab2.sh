#!/bin/bash
# round 6: gn_bwd_apply_parts grid sweep (kbench dgrad + GN backward at 96^3), in-tree vs libu3d_ab.so
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06ab2; mkdir -p $O; cd $R
for r in 1 2; do
for w in 256 512 1024 2048; do echo "== WGS $w" >> $O/kb.log; U3D_GN_APPLY_PARTS_WGS=$w timeout -k 10 100 python tools/kbench.py gnb96f >> $O/kb.log 2>&1 || exit 1; done
echo "== two-launch" >> $O/kb.log; U3D_GN_APPLY_PARTS=0 timeout -k 10 100 python tools/kbench.py gnb96f >> $O/kb.log 2>&1 || exit 1
done
grep -v amdgpu $O/kb.log
