#!/bin/bash
# round 6: small-volume conv workgroup target (U3D_SMALL_WGS, default 256) at 12^3 / 6^3
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06ff; mkdir -p $O; cd $R
for r in 1 2; do for v in 64 128 256 384 512; do echo "== SMALL_WGS=$v" >> $O/kb.log; U3D_SMALL_WGS=$v timeout -k 10 150 python tools/kbench.py fwd12 fwd6 dgrad12 dgrad6 >> $O/kb.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/kb.log
