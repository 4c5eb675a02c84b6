#!/bin/bash
# Kernel stats of the bench with / without the brick dgrad GN-backward partials.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_bgprof
mkdir -p $O
for b in 1 0; do
  (cd /tmp && export TMPDIR=/tmp && U3D_BRICK_DGRAD_GN=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$b -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-roofline > $O/kt$b.log 2>&1) || exit 1
done
