#!/bin/bash
# r04 baseline on one box: new data / DDP tests, default bench line (no CPU leg), kernel-trace profile + summary
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_base
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_data.py tests/test_gpu_ddp.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json; cut -c1-3000 $O/bench.json
timeout -k 10 200 python bench.py --no-cpu --no-infer --no-roofline --force-buckets > $O/bench_fb.log 2>&1 || { echo "bench fb failed"; tail -5 $O/bench_fb.log; exit 1; }
grep '^{' $O/bench_fb.log | tail -1 | cut -c1-300
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 13 > $O/kernel_summary.txt 2>&1 || true
head -45 $O/kernel_summary.txt
