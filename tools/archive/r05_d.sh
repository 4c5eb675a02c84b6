#!/bin/bash
# Round 5 batch: tests of every new path, step A/B (all round-5 fusions off vs on), bucket plans of the forced-bucket
# step, kernel trace of the default line.   Usage: tools/r05_d.sh TAG
TAG=${1:-r05_d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_epi_stats.py tests/test_gpu_gnfused_small.py tests/test_gpu_s2ring.py tests/test_gpu_graph.py tests/test_gpu_ddp.py tests/test_gpu_gnfused_brick.py tests/test_gpu_gnfused.py tests/test_gpu_wgrad_dma.py tests/test_gpu_slabsum.py -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|err |bitwise" $O/pytest.log | cut -c1-220
[ $rc -eq 0 ] || { grep -E "^E |Error" $O/pytest.log | head -40; exit 1; }
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
OFF="U3D_STEM_STATS=0 U3D_UP_STATS=0 U3D_SMALL_FUSE=0 U3D_FUSED_FINALIZE=0 U3D_SMALL_GB=0 U3D_S2_RING=0"
for i in 1 2 3; do
  run off$i "$OFF" || exit 1
  run on$i "A=1" || exit 1
  run slab$i "U3D_EAGER_SLAB_SUM=1" || exit 1
done
run s2off "U3D_S2_RING=0" || exit 1
run fb25_25 "A=1" --force-buckets --bucket-mb 25 --tail-mb 25 || exit 1
run fb40_2 "A=1" --force-buckets --bucket-mb 40 --tail-mb 2 || exit 1
run fb100 "A=1" --force-buckets --bucket-mb 100 --tail-mb 100 || exit 1
run plain "A=1" || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed > $O/bench_kt.log 2>&1) || { echo "prof failed"; tail -20 $O/bench_kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 16 > $O/kernel_summary.txt 2>&1 || true
head -30 $O/kernel_summary.txt
