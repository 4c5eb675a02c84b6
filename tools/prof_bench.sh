#!/bin/bash
# Kernel-trace profile of the (graph-replayed) bench: tools/prof_bench.sh TAG [bench args]
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --graph "$@" > $O/bench_kt.log 2>&1
rc=$?
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
tail -1 $O/bench_kt.log | cut -c1-200
exit $rc
