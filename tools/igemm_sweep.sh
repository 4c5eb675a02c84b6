#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for cfg in "X=0" "U3D_IGEMM_TARGET=256" "U3D_IGEMM_TARGET=1024" "U3D_IGEMM_NS=1" "U3D_IGEMM_BN=64" "U3D_IGEMM_BN=64 U3D_IGEMM_TARGET=1024" "U3D_IGEMM_BN=32"; do
  echo "== $cfg"; env $cfg timeout -k 10 100 python tools/kbench.py fwd_s2_96 fwd_s2_48 fwd_s2_24 fwd_s2_12 2>&1 | grep -v amdgpu.ids || exit 1
done
