#!/bin/bash
# Kernel-level A/B on one box: tools/kab.sh TAG ROUNDS case... -> kbench of the in-tree lib (A) and libu3d_ab.so (B),
# interleaved ROUNDS times (isolated hipGraph-replayed launches; us per launch)
TAG=$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for i in $(seq $N); do
  for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
    echo "== ${L:+B (libu3d_ab)}${L:-A (in-tree)}" >> $O/kab.log
    U3D_LIB=$L timeout -k 10 300 python tools/kbench.py "$@" >> $O/kab.log 2>&1 || exit 1
  done
done
cat $O/kab.log | grep -v amdgpu.ids
