#!/bin/bash
# r03: packed-FMA stem (tests, kernel and step A/B vs HEAD's libu3d_ab.so); GN-forward ring weight steps in
# registers 16 vs 12 (libu3d_kr.so = this tree built with -DU3D_RING_GN_KR=12)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03k
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py -k 'stem or wgrad' > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/kab.sh r03k/kab 3 stem96 wgrad_s2_96 wgrad_s2_48 wgrad_s2_24 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python tools/kbench.py fwd96_nores fwd96 2>&1 | grep -v amdgpu.ids | sed 's/^/KR16 /' | tee -a $O/kr.log || exit 1
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_kr.so timeout -k 10 300 python tools/kbench.py fwd96_nores fwd96 2>&1 | grep -v amdgpu.ids | sed 's/^/KR12 /' | tee -a $O/kr.log || exit 1
done
bash tools/ab.sh r03k/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
bash tools/ab.sh r03k/abkr "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_kr.so" 3 || exit 1
# stride-2 3^3 kernels at 2 x 96^3 / 48^3 in isolation + one SQ pass (what bounds them)
timeout -k 10 300 python tools/kbench.py fwd_s2_96 dgrad_s2_96 wgrad_s2_96 fwd_s2_48 dgrad_s2_48 wgrad_s2_48 2>&1 | grep -v amdgpu.ids | tee $O/s2.log || exit 1
bash tools/pmc_sq.sh r03k/pmc_s2 fwd_s2_96 dgrad_s2_96 wgrad_s2_96 || exit 1
python3 tools/pmc_summary.py $O/pmc_s2/run_counter_collection.csv | tee $O/pmc_s2.txt
