#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02am; mkdir -p $O
C="dec24_c1 dec24_c2 ddec24_c1 ddec24_c2 dec48_c1 ddec48_c1 dec12_c1 dec12_c2 fwd24 dgrad24"
for cfg in "X=0" "KB_SET=BRICK_MIN_WG=0" "KB_SET=SMALL_MAX_VOX=1e9" "KB_SET=BRICK_MIN_WG=0 U3D_CONVG_CO32=1" "KB_SET=USE_GEN_BRICK=0,SMALL_MAX_VOX=0"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py $C 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
