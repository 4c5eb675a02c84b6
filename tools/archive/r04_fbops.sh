#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_fbops
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/fb_ops.py > $O/fb.txt 2>&1 || { tail -20 $O/fb.txt; exit 1; }
timeout -k 10 200 python -u tools/fb_ops.py --plain > $O/plain.txt 2>&1 || { tail -20 $O/plain.txt; exit 1; }
grep -v amdgpu.ids $O/fb.txt | tail -42
echo ====
grep -v amdgpu.ids $O/plain.txt | tail -20
