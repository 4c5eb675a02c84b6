#!/bin/bash
# r04 baseline on one box: default bench line (no CPU leg), then a kernel-trace profile of the eager bench + summary
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_base
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-400
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 13 > $O/kernel_summary.txt 2>&1 || true
head -45 $O/kernel_summary.txt
