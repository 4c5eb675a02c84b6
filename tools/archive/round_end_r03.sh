#!/bin/bash
# Round-3 closing measurements on one box: whole GPU suite, smoke(), PMC traffic + SQ pass of the dominant kernel,
# default bench line (with the CPU baseline, before the counter passes), kernel-trace profile of the bench (--no-roofline) + per-kernel summary,
# a second trace WITH the standalone roofline launches for the event-vs-trace timing check.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_end
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
# the bench line runs before the PMC passes: the first run after a counter pass measured 8.1 vs 6.0 ms/step on the
# same box (profiles/r03_benchvar.log)
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
bash tools/pmc_conv32.sh profiles/r03_pmc_conv32_fwd.json > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
cp profiles/r03_pmc_conv32_fwd.json $O/
bash tools/pmc_sq.sh r03_end_sq fwd96 > $O/sq.log 2>&1 || { echo "sq failed"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r03_end_sq/run_counter_collection.csv > $O/sq_summary.txt 2>&1 || true
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 13 > $O/kernel_summary.txt 2>&1 || true
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt2 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $O/bench_kt2.log 2>&1) || { echo "prof2 failed"; exit 1; }
python3 tools/timing_check.py $O/kt2 $O/bench_kt2.log 10 profiles/r03_conv32_timing_check.json > $O/timing.log 2>&1 || { echo "timing check failed"; tail -5 $O/timing.log; }
cp profiles/r03_conv32_timing_check.json $O/ 2>/dev/null
head -25 $O/kernel_summary.txt
cut -c1-600 $O/bench.json
