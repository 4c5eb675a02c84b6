#!/bin/bash
# round 6: head backward load look-ahead (ND tiles in flight): in-tree ND=3 vs ND=2 / ND=4 builds; head tests
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06q; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_head_loss.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do for L in "" v_nd2 v_nd4; do echo "== ${L:-nd3}" >> $O/kb.log; U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/$L.so} timeout -k 10 120 python tools/kbench.py hlb96plain hlb96gn hlb96sep hlb96fused >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
