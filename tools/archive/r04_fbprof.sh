#!/bin/bash
# r04: host (Python) time of the plain and the forced-bucket bench step: cProfile over 10 eager steps, top functions
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_fbprof
mkdir -p $O
cd $R
for m in plain fb; do
  a=""; [ $m = fb ] && a="--force-buckets"
  timeout -k 10 300 python -m cProfile -o $O/$m.prof bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer $a > $O/bench_$m.log 2>&1 || { tail -5 $O/bench_$m.log; exit 1; }
  grep '^{' $O/bench_$m.log | cut -c1-200
  python -c "
import pstats; p = pstats.Stats('$O/$m.prof'); p.sort_stats('tottime').print_stats(30)" > $O/top_$m.txt 2>&1
  python -c "
import pstats; p = pstats.Stats('$O/$m.prof'); p.sort_stats('cumulative').print_stats(40)" > $O/cum_$m.txt 2>&1
done
