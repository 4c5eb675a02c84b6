#!/bin/bash
# copy the round-4 closing measurements (gpurun_out/r04_end) into profiles/ (committed evidence)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r04_end
P=$R/profiles
cp $O/kernel_summary.txt $P/r04_kernel_summary.txt
cp $O/bench.json $P/r04_bench.json
cp $O/bench_fb.json $P/r04_bench_force_buckets.json
cp $O/pytest.log $P/r04_gpu_pytest.log
cp $O/smoke.log $P/r04_smoke.log
for t in wgrad96 dgrad96gn fwd96; do [ -f $O/pmc_$t.json ] && cp $O/pmc_$t.json $P/r04_pmc_$t.json; done
for t in wgrad96 dgrad96gn; do [ -f $O/sq_$t.txt ] && cp $O/sq_$t.txt $P/r04_pmc_sq_$t.txt; done
python3 $R/tools/gap_summary.py $O/run_kernel_trace.csv > $P/r04_step_gaps.txt || true
ls -la $P/r04_*
