#!/bin/bash
# r06 first call: data-parallel / graph tests after the used-flag + capture-condition changes, then the ring ablation
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_a; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_ddp.py tests/test_gpu_graph.py > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for L in "" libu3d_abl1.so libu3d_abl2.so libu3d_abl3.so; do
  echo "== lib ${L:-in-tree}" >> $O/kb.log
  U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/$L} timeout -k 10 200 python tools/kbench.py fwd96 fwd96nr dgrad96gn wgrad96 wgrad96nogn >> $O/kb.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/kb.log
