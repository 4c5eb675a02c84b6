#!/bin/bash
# r04: LDS-DMA weight-gradient ring: parity (bitwise vs the register ring, fp64), stamps, kernel + step A/B (U3D_WR_DMA)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_b
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad_dma.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -k "wgrad or ring" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in wgrad96 wgrad48; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c 2.5 >> $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
done
grep -v amdgpu.ids $O/stamps.txt
for i in 1 2; do
  for v in 1 0; do
    echo "== U3D_WR_DMA=$v" >> $O/kab.log
    U3D_WR_DMA=$v timeout -k 10 120 python tools/kbench.py wgrad96 wgrad48 >> $O/kab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/kab.log
bash tools/ab.sh r04_b/ab "U3D_WR_DMA=1" "U3D_WR_DMA=0" 3
bash tools/r04_fb.sh
