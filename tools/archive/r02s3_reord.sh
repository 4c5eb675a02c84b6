#!/bin/bash
# Default-path check after the epilogue loop reorder (tn outer): micro-benchmarks and step A/B vs the previous build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_reord
mkdir -p $O
cd $R
timeout -k 10 120 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 2>/dev/null | tee $O/kbench.log || exit 1
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so timeout -k 10 120 python tools/kbench.py fwd48 dgrad48 fwd24 dgrad24 2>/dev/null | sed 's/^/prev: /' | tee -a $O/kbench.log || exit 1
bash tools/ab.sh r02s3_reord/ab "U3D_NONE=0" "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_ab.so" 3 || exit 1
