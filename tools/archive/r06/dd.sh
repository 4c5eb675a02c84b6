#!/bin/bash
# round 6: stem weight gradient with 1 / 2 / 3 bricks staged per load round: tests (in-tree BP=2), kbench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06dd; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bf16.py -k "stem" tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do for L in "" v_bp1 v_bp3; do echo "== ${L:-bp2}" >> $O/kb.log; U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/$L.so} timeout -k 10 120 python tools/kbench.py stemw96 >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
