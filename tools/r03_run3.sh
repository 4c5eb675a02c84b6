#!/bin/bash
# r03: packed-FMA stem (tests, kernel and step A/B vs HEAD's libu3d_ab.so); GN-forward ring weight steps in
# registers 16 vs 12 (libu3d_kr.so = this tree built with -DU3D_RING_GN_KR=12)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03k
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py -k stem > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03k/kab 3 stem96 fwd96_nores || exit 1
for i in 1 2 3; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_kr.so timeout -k 10 300 python tools/kbench.py fwd96_nores fwd96 2>&1 | grep -v amdgpu.ids | sed 's/^/KR12 /' | tee -a $O/kr.log || exit 1
done
bash tools/ab.sh r03k/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
bash tools/ab.sh r03k/abkr "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_kr.so" 3 || exit 1
