#!/bin/bash
# Round 5 batch f: per-site finalize micro-A/B, slab sum, kernel trace with the in-launch finalize off.
TAG=${1:-r05_f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/r05_fin.py > $O/fin.log 2>&1 || { echo "fin failed"; tail -20 $O/fin.log; exit 1; }
cat $O/fin.log
(cd /tmp && export TMPDIR=/tmp U3D_FUSED_FINALIZE=0 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed > $O/bench_kt.log 2>&1) || { echo "prof failed"; tail -20 $O/bench_kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 16 > $O/kernel_summary.txt 2>&1 || true
head -45 $O/kernel_summary.txt
timeout -k 10 120 python tools/kbench.py fwds2ring > $O/kb_s2.log 2>&1 && cat $O/kb_s2.log
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py s2ring96 > $O/stamps_s2.log 2>&1; cat $O/stamps_s2.log | tail -12
