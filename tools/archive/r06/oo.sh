#!/bin/bash
# round 6: 1^3 weight gradient with 1024-voxel chunks (libu3d_w1k) vs 512 (tree): kbench 3 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06oo; mkdir -p $O; cd $R
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_w1k.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_bf16.py -k "1x1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for V in tree w1k; do
  echo "== $V" >> $O/kb.log
  L=""; [ $V = w1k ] && L=$R/multimodal-pl_amd/u3d/libu3d_w1k.so
  U3D_LIB=$L timeout -k 10 120 python tools/kbench.py wgrad1_96 wgrad1_s2_96 >> $O/kb.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/kb.log | paste - - -
