#!/bin/bash
# GPU check used with gpurun: tests, bench, kernel-trace profile. Usage: tools/gpu_check.sh TAG [tests|bench|prof ...]
# Stops at the first crash/timeout (exit code other than 0 or a plain test failure).
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 -a "$2" = tests ]; }
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python -m pytest $R/tests -m gpu -x -q > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log ;;
    bench) timeout -k 10 400 python $R/bench.py > $O/bench.log 2>&1; rc=$?; tail -2 $O/bench.log ;;
    benchq) timeout -k 10 300 python $R/bench.py --no-cpu > $O/bench.log 2>&1; rc=$?; tail -2 $O/bench.log ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $O/bench_kt.log 2>&1); rc=$?
          f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/kt/ 2>/dev/null; tail -1 $O/bench_kt.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step rc=$rc"
  ok $rc $step || exit $rc
done
