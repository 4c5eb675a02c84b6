#!/bin/bash
# Round-4 closing measurements on one box (committed under profiles/r04_*): whole GPU suite, smoke(), the default bench
# line (with the CPU baseline and the configs[4] leg, before any counter pass), the forced-bucket line, a kernel-trace
# profile of the bench + summary (the roofline's trace check reads it), PMC traffic and an SQ pass of the three 96^3
# ring kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_end
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json; cut -c1-300 $O/bench.json
timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --force-buckets > $O/bench_fb.log 2>&1 || { echo "fb failed"; exit 1; }
grep '^{' $O/bench_fb.log | tail -1 > $O/bench_fb.json; cut -c1-200 $O/bench_fb.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu --no-roofline --no-infer --eager > $O/bench_kt.log 2>&1) || { echo "prof failed"; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && cp $(dirname $f)/*.csv $O/
python3 tools/prof_summary.py $O 13 > $O/kernel_summary.txt 2>&1 || true
head -25 $O/kernel_summary.txt
bash tools/pmc_ring.sh wgrad96 "wgrad_ring" $O/pmc_wgrad96.json > $O/pmc1.log 2>&1 || { echo "pmc1 failed"; exit 1; }
bash tools/pmc_ring.sh dgrad96gn "conv32_ring_kernel<true, true, false" $O/pmc_dgrad96gn.json > $O/pmc2.log 2>&1 || { echo "pmc2 failed"; exit 1; }
bash tools/pmc_ring.sh fwd96 "conv32_ring_kernel<false, true, true" $O/pmc_fwd96.json > $O/pmc3.log 2>&1 || { echo "pmc3 failed"; exit 1; }
for c in wgrad96 dgrad96gn; do
  bash tools/pmc_sq.sh r04_end_sq_$c $c > /dev/null 2>&1 || { echo "sq $c failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/r04_end_sq_$c/run_counter_collection.csv > $O/sq_$c.txt 2>&1
done
cat $O/pmc_*.json
