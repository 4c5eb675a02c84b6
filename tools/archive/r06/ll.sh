#!/bin/bash
# round 6: where the conv1 weight gradient's 46 us go: timing-only ablation builds (sw1 = one MFMA step per brick,
# sw2 = only the ci = 0 slab column stored, sw3 = both) against the tree, kbench 3 rounds; then SQ passes of the tree
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06ll; mkdir -p $O; cd $R
for i in 1 2 3; do for L in "" sw1 sw2 sw3; do
  echo "== ${L:-tree}" >> $O/kb.log
  U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/libu3d_$L.so} timeout -k 10 120 python tools/kbench.py stemw96 >> $O/kb.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/kb.log | paste - - 
bash tools/pmc_sq2.sh r06ll/sq stemw96 && echo pmc ok
