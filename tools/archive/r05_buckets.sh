#!/bin/bash
# Round 5: bucket plans of the graph-captured forced-bucket step vs the plain line, alternating on one box.
TAG=${1:-r05_buckets}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for i in 1 2; do
  for cfg in "plain" "--force-buckets --bucket-mb 25 --tail-mb 25" "--force-buckets --bucket-mb 40 --tail-mb 2" "--force-buckets --bucket-mb 25 --tail-mb 2" "--force-buckets --bucket-mb 34 --tail-mb 34" "--force-buckets --bucket-mb 100 --tail-mb 100"; do
    a=$cfg; [ "$cfg" = plain ] && a=""
    tag=$(echo "$cfg" | tr -d ' -')
    timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 $a > $O/bench_$i$tag.log 2>&1 || { echo "bench $cfg failed"; grep -v "^frame" $O/bench_$i$tag.log | tail -20; exit 1; }
    grep '^{' $O/bench_$i$tag.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['launch'], d.get('graph_error'))"
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed --force-buckets > $O/bench_kt.log 2>&1) || { echo "prof failed"; tail -20 $O/bench_kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
