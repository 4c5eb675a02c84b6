#!/bin/bash
# r04: stem weight gradient with a two-deep register prefetch (in-tree) vs HEAD (libu3d_ab.so); parity first
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_y
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -x -q -k "stem" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py stemw96 stem96 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
