#!/bin/bash
# Round 5 batch l: weight LDS fill with all loads in flight (ring, stride-2 ring), 256-thread brick GN finalize:
# parity, kernel A/B against the previous library, stamps, step A/B.
TAG=${1:-r05_l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_epi_stats.py tests/test_gpu_s2ring.py tests/test_gpu_gnfused.py tests/test_gpu_pbrick.py tests/test_gpu_fullsize.py -k "ring or s2 or stats or fused or pbrick or trunk_conv" -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -cE "PASSED" $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $O/pytest.log | head -30; exit 1; }
timeout -k 10 120 python tools/kbench.py fwd96 fwd96_nores dgrad96gn fwd48st fwds2ring > $O/kb.log 2>&1; grep -v amdgpu.ids $O/kb.log
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_prev.so timeout -k 10 120 python tools/kbench.py fwd96 fwd96_nores dgrad96gn fwd48st fwds2ring > $O/kb_prev.log 2>&1; grep -v amdgpu.ids $O/kb_prev.log | sed 's/^/prev /'
for c in fwdnores96 dgradgn96; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c > $O/stamps_$c.log 2>&1; echo "== $c"; grep -v amdgpu.ids $O/stamps_$c.log | head -6
done
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run new$i "A=1" || exit 1
  run prev$i "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_prev.so" || exit 1
done
