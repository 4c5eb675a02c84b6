#!/bin/bash
# Round-2 closing measurements on the final tree (session 3, after the slab-sum change): GPU suite, PMC traffic of the dominant kernel, default
# bench line (with the CPU baseline), a kernel-trace profile of the bench without the standalone roofline launches,
# a second trace with them for the event-vs-trace timing check, smoke().
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02_end6
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "tests failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/pmc_conv32.sh gpurun_out/r02_end6/pmc_conv32_fwd.json > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt2 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $O/bench_kt2.log 2>&1) || { echo "prof2 failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); cp $f $O/run_kernel_trace.csv
python tools/prof_summary.py $O 13 > $O/kernel_summary.txt || true
python tools/timing_check.py $O/kt2 $O/bench_kt2.log 10 $O/conv32_timing_check.json > $O/timing.log 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
head -3 $O/kernel_summary.txt
cut -c1-400 $O/bench.json
