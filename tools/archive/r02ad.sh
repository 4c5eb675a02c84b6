#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "brick or convg or trunk or gn or block or g3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "U3D_CONVG_CO32=0" "U3D_CONVG_CO32=-1" "U3D_CONVG_CO32=1"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 fwd12 dgrad12 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
bash tools/ab.sh r02ad "U3D_LIB=$R/tools/ab_lib/libu3d_a.so" "U3D_LIB=" 3
