#!/bin/bash
# r06: weight-gradient ring workgroup target (slab count) per level: kernel + slab-sum time at WR_WGS 256 / 192 / 128
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_n; mkdir -p $O; cd $R
for r in 1 2; do for v in 256 192 128 96; do echo "== WR_WGS=$v" >> $O/kb.log; U3D_WR_WGS=$v timeout -k 10 120 python tools/kbench.py wgrad48 wgrad24 wgrad12 wgsum48 wgsum24 wgsum12 >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
