#!/bin/bash
# Tree check on one box: whole GPU suite, smoke(), default bench line, kernel-trace profile of the bench.
# tools/r03_check.sh TAG
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
bash tools/prof_bench.sh $TAG > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O 13 > $O/kernel_summary.txt 2>&1 || true
head -25 $O/kernel_summary.txt
