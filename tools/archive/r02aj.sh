#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02aj; mkdir -p $O
for cfg in "X=0" "KB_SET=GN_MATERIALIZE_MIN_C=32,GN_MATERIALIZE_BYTES=1e9" "KB_SET=GN_MATERIALIZE_BYTES=1e9"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py fwd_s2_96 fwd_s2_48 fwd_s2_24 fwd_s2_12 gnapply96 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
