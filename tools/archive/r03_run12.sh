#!/bin/bash
# r03: conv1 stem, one voxel per lane (U3D_STEM1=2) vs four (1)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03v
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py -k stem > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for v in 1 2; do echo "STEM1=$v" >> $O/k.log; U3D_STEM1=$v timeout -k 10 200 python tools/kbench.py stem96 2>&1 | grep -v amdgpu.ids >> $O/k.log || exit 1; done; done
cat $O/k.log
bash tools/ab.sh r03v/ab "U3D_STEM1=1" "U3D_STEM1=2" 3 || exit 1
