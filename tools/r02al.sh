#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02al; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_epistats.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "stem or g3 or bf16_training" > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
for cfg in "U3D_STEM_MFMA=0" "U3D_STEM_MFMA=1"; do
  echo "== $cfg" | tee -a $O/k.txt
  env $cfg timeout -k 10 100 python tools/kbench.py stem96 2>&1 | grep -v amdgpu.ids | tee -a $O/k.txt || exit 1
done
U3D_STEM_MFMA=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py -k stem > $O/pytest_mfma.log 2>&1 || exit 1
bash tools/ab.sh r02al "U3D_STEM_MFMA=0" "U3D_STEM_MFMA=1" 4
