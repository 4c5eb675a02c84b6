#!/bin/bash
# Round 5 batch e: batched last-arriver combines + the GN16 finalize kernel; per-feature A/B (each round-5 fusion off
# alone against all on), kernel trace of the default line.   Usage: tools/r05_e.sh TAG
TAG=${1:-r05_e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_epi_stats.py tests/test_gpu_gnfused_small.py tests/test_gpu_s2ring.py tests/test_gpu_gnfused_brick.py tests/test_gpu_gnfused.py tests/test_gpu_ddp.py tests/test_gpu_graph.py -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -cE "PASSED" $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E |Error" $O/pytest.log | head -40; exit 1; }
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run on$i "A=1" || exit 1
  run ff$i "U3D_FUSED_FINALIZE=0" || exit 1
  run sf$i "U3D_SMALL_FUSE=0" || exit 1
  run us$i "U3D_UP_STATS=0" || exit 1
  run ss$i "U3D_STEM_STATS=0" || exit 1
  run gb$i "U3D_SMALL_GB=0" || exit 1
done
run fb "A=1" --force-buckets || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed > $O/bench_kt.log 2>&1) || { echo "prof failed"; tail -20 $O/bench_kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 16 > $O/kernel_summary.txt 2>&1 || true
head -45 $O/kernel_summary.txt
