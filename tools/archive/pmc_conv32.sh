#!/bin/bash
# HBM traffic of the dominant kernel (32->32 conv fwd, GN prologue + residual, 2x96^3): two --pmc passes
# (FETCH_SIZE, WRITE_SIZE; separate runs), then tools/pmc_traffic.py. Usage: tools/pmc_conv32.sh OUT.json
OUTJ=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc32
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 $R/tools/kbench.py fwd96 > $O/f.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $R/tools/kbench.py fwd96 > $O/w.log 2>&1 || exit 1
cp $(find $O/f -name '*counter_collection.csv' | head -1) $O/fetch.csv
cp $(find $O/w -name '*counter_collection.csv' | head -1) $O/write.csv
mkdir -p $O/fd $O/wd && cp $O/fetch.csv $O/fd/run_counter_collection.csv && cp $O/write.csv $O/wd/run_counter_collection.csv
python3 $R/tools/pmc_traffic.py $O/fd $O/wd "conv32_ring_kernel<false, true, true" $R/$OUTJ 20
