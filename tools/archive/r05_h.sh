#!/bin/bash
# Round 5 batch h: stride-2 ring with the staging interleaved into the MFMA taps: parity, kernel time, stamps.
TAG=${1:-r05_h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_s2ring.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED" $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest.log | head; exit 1; }
timeout -k 10 120 python tools/kbench.py fwds2ring > $O/kb_s2.log 2>&1 && cat $O/kb_s2.log | grep -v amdgpu.ids
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py s2ring96 > $O/stamps_s2.log 2>&1; tail -12 $O/stamps_s2.log
