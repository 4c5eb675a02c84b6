#!/bin/bash
# r04: wgrad ring variants, kernel A/B (kbench, hipGraph replay): register ring with hoisted staging offsets (in-tree,
# WR_DMA=0) vs the committed register ring (libu3d_ab.so = HEAD) vs the DMA ring (lookahead 1/2/3); parity first
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_dma.py tests/test_gpu_pbrick.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_WR_DMA=0" "U3D_LIB=$L/libu3d_ab.so U3D_WR_DMA=0" "U3D_WR_DMA=1" "U3D_LIB=$L/libu3d_la2.so" "U3D_LIB=$L/libu3d_la3.so" "U3D_LIB=$L/libu3d_prio.so U3D_WR_DMA=0"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py wgrad96 wgrad48 fwd96 fwd96_nores dgrad96gn >> $O/kab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/kab.log
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1) ; grep -o "SQ_[A-Z_0-9]*" $O/counters.txt | sort -u | tr '\n' ' ' | head -c 4000
for i in 1 2; do
  for v in "U3D_IGEMM_BM=128" "U3D_IGEMM_BM=0"; do
    echo "== $v" >> $O/kab_igemm.log
    env $v timeout -k 10 120 python tools/kbench.py fwd_s2_96 fwd_s2_48 fwd_s2_24 >> $O/kab_igemm.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/kab_igemm.log
