#!/bin/bash
# Round-2 closing measurements: PMC traffic + SQ pass of the dominant kernel, default bench line (with the CPU
# baseline), a clean kernel-trace profile of the bench (--no-roofline: no standalone launches in the summary), a
# second trace WITH the standalone roofline launches for the event-vs-trace timing check, smoke().
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02_end
mkdir -p $O
cd $R
bash tools/pmc_conv32.sh profiles/r02_pmc_conv32_fwd.json > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
cp profiles/r02_pmc_conv32_fwd.json $O/
bash tools/pmc_sq.sh r02_end_sq fwd96 > $O/sq.log 2>&1 || { echo "sq failed"; exit 1; }
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt2 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $O/bench_kt2.log 2>&1) || { echo "prof2 failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cut -c1-400 $O/bench.json
