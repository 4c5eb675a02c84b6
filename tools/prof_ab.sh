#!/bin/bash
# A/B kernel-trace profile of bench.py under two environments: tools/prof_ab.sh TAG "ENV_A" "ENV_B"
TAG=$1; A=$2; B=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in a b; do
  E=$A; [ $v = b ] && E=$B
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline > $O/bench_$v.log 2>&1 || exit $?
  tail -1 $O/bench_$v.log | cut -c1-220
done
