#!/bin/bash
# Timing ablations of the persistent brick conv at 48^3 (fwd, GN + residual): 1 no MFMA, 2 no weight loads,
# 4 no halo loads, 8 no LDS staging writes, 16 no LDS fragment reads (results wrong; timing only), then an SQ pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_pbabl
mkdir -p $O
cd $R
for a in 0 1 2 6 14 16 17 31 0; do
  echo -n "abl=$a "; U3D_PB_ABL=$a timeout -k 10 120 python tools/kbench.py fwd48 2>/dev/null | grep fwd48 || exit 1
done | tee $O/abl.log
bash tools/pmc_sq.sh r02s3_pbabl/sq fwd48 dgrad48 fwd24 fwd96 || exit 1
python tools/pmc_summary.py $O/sq/*counter_collection.csv
