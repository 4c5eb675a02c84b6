#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ao; mkdir -p $O
for cfg in "KB_WGRAD=ring" "KB_WGRAD=brick" "X=0"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py wgrad96 wgrad48 wgrad24 wgrad12 wgrad6 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
