#!/bin/bash
# r04: what the forced-bucket (RCCL world 1) step pays: kernel traces of the plain and the --force-buckets bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_fb
mkdir -p $O
cd $R
for m in plain fb; do
  a=""; [ $m = fb ] && a="--force-buckets"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$m -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer $a > $O/bench_$m.log 2>&1) || { echo "prof $m failed"; tail -5 $O/bench_$m.log; exit 1; }
  mkdir -p $O/s_$m; f=$(find $O/kt_$m -name '*kernel_trace.csv' | head -1); cp $(dirname $f)/*.csv $O/s_$m/
  python3 tools/prof_summary.py $O/s_$m 13 > $O/summary_$m.txt 2>&1 || true
  grep '^{' $O/bench_$m.log | cut -c1-160
  head -3 $O/summary_$m.txt
done
