#!/bin/bash
# r04: wgrad ring variants, kernel A/B (kbench, hipGraph replay): DMA (hoisted addresses) with fragment lookahead 1/2/3
# vs the register-staged ring; bitwise test of the in-tree DMA kernel first
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_dma.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in "U3D_WR_DMA=0" "U3D_WR_DMA=1" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_la2.so" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_la3.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py wgrad96 wgrad48 >> $O/kab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/kab.log
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1) ; grep -o "SQ_[A-Z_]*" $O/counters.txt | sort -u | tr '\n' ' ' | head -c 3000
