#!/bin/bash
# Round-6 closing measurements, part 2 (committed under profiles/r06_*): the default bench line, the forced-bucket line,
# a kernel trace of the bench summarised over its 10 timed replays only (tools/trace_steps.py), PMC traffic of the three
# 96^3 ring kinds and SQ passes (whole-launch and per-pipe) of the weight-gradient and data-gradient rings.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06_end; mkdir -p $O; cd $R
PART=${1:-all}
if [ "$PART" = all ] || [ "$PART" = prof ]; then
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --no-mixed > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 10 40 steady > $O/kernel_summary.txt 2>&1 || true
head -24 $O/kernel_summary.txt
python3 tools/trace_stats.py $O 10 steady > $O/trace_stats.txt 2>&1; head -3 $O/trace_stats.txt
bash tools/pmc_ring.sh wgrad96 "wgrad_ring_dma_kernel<true>" $O/pmc_wgrad96.json > $O/pmc1.log 2>&1 || { echo "pmc1 failed"; exit 1; }
bash tools/pmc_ring.sh dgrad96gn "conv32_ring_kernel<true, true, false" $O/pmc_dgrad96gn.json > $O/pmc2.log 2>&1 || { echo "pmc2 failed"; exit 1; }
bash tools/pmc_ring.sh fwd96 "conv32_ring_kernel<false, true, true" $O/pmc_fwd96.json > $O/pmc3.log 2>&1 || { echo "pmc3 failed"; exit 1; }
for c in wgrad96 dgrad96gn; do
  bash tools/pmc_sq.sh r06_end_sq_$c $c > /dev/null 2>&1 || { echo "sq $c failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/r06_end_sq_$c/run_counter_collection.csv > $O/sq_$c.txt 2>&1
done
bash tools/pmc_sq2.sh r06_end_sq2 fwd96 dgrad96gn wgrad96 > /dev/null 2>&1 || { echo "sq2 failed"; exit 1; }
for p in a b; do python3 tools/pmc_summary.py gpurun_out/r06_end_sq2/${p}_counter_collection.csv >> $O/sq2.txt 2>&1; done
cat $O/pmc_*.json
# the bench line's trace_check reads the newest profiles/*kernel_summary.txt: the trace just taken on this box
cp $O/kernel_summary.txt profiles/r06_kernel_summary.txt
fi
if [ "$PART" = all ] || [ "$PART" = bench ]; then
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json; cut -c1-400 $O/bench.json
timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --force-buckets > $O/bench_fb.log 2>&1 || { echo "fb failed"; exit 1; }
grep '^{' $O/bench_fb.log | tail -1 > $O/bench_fb.json; cut -c1-200 $O/bench_fb.json
fi
