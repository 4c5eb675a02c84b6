#!/bin/bash
# HBM traffic of one kbench case's kernel: two --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs), then
# tools/pmc_traffic.py.  Usage: tools/pmc_ring.sh CASE "KERNEL-SUBSTRING" OUT.json
#   e.g. tools/pmc_ring.sh wgrad96 "wgrad_ring_kernel<true, 16, 16>" profiles/r04_pmc_wgrad96.json
CASE=$1; KRX=$2; OUTJ=$3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$CASE
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 $R/tools/kbench.py $CASE > $O/f.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $R/tools/kbench.py $CASE > $O/w.log 2>&1 || exit 1
mkdir -p $O/fd $O/wd
cp $(find $O/f -name '*counter_collection.csv' | head -1) $O/fd/run_counter_collection.csv
cp $(find $O/w -name '*counter_collection.csv' | head -1) $O/wd/run_counter_collection.csv
case "$OUTJ" in /*) OJ=$OUTJ;; *) OJ=$R/$OUTJ;; esac
python3 $R/tools/pmc_traffic.py $O/fd $O/wd "$KRX" $OJ 20
