#!/bin/bash
# r04: full GPU suite, then the default bench line, the forced-bucket (RCCL world 1) line x2 alternating with the plain
# one, and a kernel-trace summary of the default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_d
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --no-cpu > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json; cut -c1-400 $O/bench.json
for i in 1 2; do
  for a in "" "--force-buckets"; do
    ms=$(timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 $a 2>>$O/fb.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "plain${a} $ms" | tee -a $O/fb.log
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 13 > $O/kernel_summary.txt 2>&1 || true
head -30 $O/kernel_summary.txt
