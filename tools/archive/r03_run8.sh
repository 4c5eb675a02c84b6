#!/bin/bash
# r03: ring conv on v_mfma_f32_16x16x32_bf16 (in-tree) vs 32x32x16 (libu3d_ab.so, -DU3D_RING_M16=0); slab-cap A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03q
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_queue.py -k "ring or conv32 or step or queue" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03q/kab 2 fwd96 fwd96_nores dgrad96 || exit 1
bash tools/ab.sh r03q/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
for cap in 0 8192 2048; do
  echo "cap=$cap" >> $O/k.log
  U3D_WG_SLAB_KB=$cap timeout -k 10 200 python tools/kbench.py wgrad12 wgrad6 wgrad24 2>&1 | grep -v amdgpu.ids >> $O/k.log || exit 1
done
cat $O/k.log
bash tools/ab.sh r03q/ab1 "U3D_WG_SLAB_KB=0" "U3D_WG_SLAB_KB=8192" 3 || exit 1
