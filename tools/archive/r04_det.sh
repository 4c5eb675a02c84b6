#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_det3
mkdir -p $O
cd $R
timeout -k 10 150 python -u tools/path_diff.py > $O/held.log 2>&1 || { tail -20 $O/held.log; exit 1; }
PD_HOLD=0 timeout -k 10 150 python -u tools/path_diff.py > $O/polled.log 2>&1 || { tail -20 $O/polled.log; exit 1; }
grep -v amdgpu.ids $O/held.log | head -150
echo =====
grep -v amdgpu.ids $O/polled.log | head -60
