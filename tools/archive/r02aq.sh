#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 200 python tools/host_time.py 20 2>&1 | grep -v amdgpu.ids
