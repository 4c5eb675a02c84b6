#!/bin/bash
# r03: conv1 stem with a scalar-loaded weight table; stride-2 wgrad halo parity split; stride-2 dgrad transposed
# MFMA with a register epilogue (libu3d_ab.so = HEAD: everything but the dgrad change)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03l
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py -k 'stem or wgrad or dgrad' > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/kbench.py stem96 wgrad_s2_96 wgrad_s2_48 wgrad_s2_24 2>&1 | grep -v amdgpu.ids | tee $O/k1.log || exit 1
bash tools/kab.sh r03l/kab 2 dgrad_s2_96 dgrad_s2_48 dgrad_s2_24 dgrad_s2_12 || exit 1
bash tools/pmc_sq.sh r03l/pmc_s2 wgrad_s2_96 dgrad_s2_96 || exit 1
python3 tools/pmc_summary.py $O/pmc_s2/run_counter_collection.csv | grep -A2 "wgrad_brick\|dgrad_s2" | tee $O/pmc_s2.txt
bash tools/ab.sh r03l/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 2 || exit 1
