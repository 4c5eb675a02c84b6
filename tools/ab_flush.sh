#!/bin/bash
# A/B of the side-stream weight-gradient flush (U3D_SIDE_FLUSH) on the default bench. Usage: tools/ab_flush.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for v in 0 4 8 0 4 8; do
  U3D_SIDE_FLUSH=$v timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 > $O/b_$v.log 2>&1 || exit 1
  echo "flush=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b_$v.log)"
done
