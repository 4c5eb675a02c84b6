#!/bin/bash
# round 6: GroupNorm apply with ACC templated, GA_U voxels per round (in-tree U=2; v_ga1 / v_ga4) vs libu3d_ab.so
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06hh; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_gnfused.py tests/test_gpu_conv1x1.py tests/test_gpu_head_loss.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do for L in "" v_ga1 v_ga4 libu3d_ab; do echo "== ${L:-ga2}" >> $O/kb.log; U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/$L.so} timeout -k 10 120 python tools/kbench.py gnbwd96 gnbwd2s96 gnb96f gnbwd48 >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
