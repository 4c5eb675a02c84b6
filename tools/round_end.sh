#!/bin/bash
# Round-closing measurements on the GPU box: PMC traffic of the dominant kernel, default bench line (with the CPU
# baseline), kernel-trace profile of the bench, smoke(). Usage: tools/round_end.sh TAG   (outputs: gpurun_out/TAG)
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
bash $R/tools/pmc_conv32.sh profiles/${TAG}_pmc_conv32_fwd.json > $O/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
cp $R/profiles/${TAG}_pmc_conv32_fwd.json $O/
cd $R && timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
cut -c1-300 $O/bench.json
