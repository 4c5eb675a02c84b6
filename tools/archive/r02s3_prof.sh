#!/bin/bash
# Kernel-trace profile of the eager bench on the current tree (no standalone roofline launches): per-kernel step summary.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s3_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline > $O/bench_kt.log 2>&1 || { tail -5 $O/bench_kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); cp $(dirname $f)/*.csv $O/
cd $R && python tools/prof_summary.py $O 13 > $O/summary.txt && head -45 $O/summary.txt
grep '^{' $O/bench_kt.log | cut -c1-300
