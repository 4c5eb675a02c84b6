#!/bin/bash
# round 6: head grid sweep (plain backward, forward, GN-partials backward)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06p; mkdir -p $O; cd $R
for nb in 512 768 1024 1536 2048; do echo "== HEAD_NB=$nb" >> $O/kb.log; U3D_HEAD_NB=$nb timeout -k 10 120 python tools/kbench.py hlb96plain head96 hlb96plain head96 >> $O/kb.log 2>&1 || exit 1; done
for nb in 256 512 1024 1536; do echo "== HEAD_GN_NB=$nb" >> $O/kb.log; U3D_HEAD_GN_NB=$nb timeout -k 10 120 python tools/kbench.py hlb96gn hlb96gn >> $O/kb.log 2>&1 || exit 1; done
grep -v amdgpu $O/kb.log
