#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_epistats.py -k "gn or GN or stats or block or g3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
A=$R/tools/ab_lib/libu3d_a.so
for lib in $A "" $A ""; do
  echo "== lib=${lib:-new}" | tee -a $O/gn.txt
  U3D_LIB=$lib bash tools/gn_prof.sh r02ab_tmp > /dev/null || exit 1
  cat gpurun_out/r02ab_tmp/gn.txt | tr '\n' ' ' | sed 's/ *0.0 TFLOP\/s//g' | tee -a $O/gn.txt; echo | tee -a $O/gn.txt
done
bash tools/ab.sh r02ab "U3D_LIB=$A" "U3D_LIB=" 3
