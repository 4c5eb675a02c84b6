#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_host
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/host_prof.py > $O/prof.txt 2>&1 || { tail -30 $O/prof.txt; exit 1; }
grep -v amdgpu.ids $O/prof.txt | head -5
