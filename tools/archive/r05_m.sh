#!/bin/bash
# Round 5 batch m: progress priority in the 96^3 ring loops (U3D_PPRIO, compile-time; libu3d_nopp.so = the same tree
# without it): parity, stamps, kernel and step A/B.
TAG=${1:-r05_m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_epi_stats.py tests/test_gpu_gnfused.py tests/test_gpu_wgrad_dma.py tests/test_gpu_fullsize.py -k "ring or stats or fused or dma or trunk_conv" -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -cE "PASSED" $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|^E " $O/pytest.log | head -30; exit 1; }
timeout -k 10 120 python tools/kbench.py fwd96 fwd96_nores dgrad96gn wgrad96 wgrad48 > $O/kb.log 2>&1; grep -v amdgpu.ids $O/kb.log
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_nopp.so timeout -k 10 120 python tools/kbench.py fwd96 fwd96_nores dgrad96gn wgrad96 wgrad48 > $O/kb_nopp.log 2>&1; grep -v amdgpu.ids $O/kb_nopp.log | sed 's/^/nopp /'
for c in fwdnores96 dgradgn96 wgrad96; do
  U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_stamps.so timeout -k 10 120 python tools/stamps.py $c > $O/stamps_$c.log 2>&1; echo "== $c"; grep -v amdgpu.ids $O/stamps_$c.log | sed -n '3,5p;6p;10p'
done
run() {  # run TAG ENV ARGS
  local t=$1; shift; local e=$1; shift
  env $e timeout -k 10 300 python bench.py --no-cpu --no-infer --no-roofline --no-mixed --steps 30 --warmup 5 "$@" > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; grep -v "^frame" $O/bench_$t.log | tail -20; exit 1; }
  grep '^{' $O/bench_$t.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['launch'], d.get('graph_error'))"
}
for i in 1 2; do
  run pp$i "A=1" || exit 1
  run nopp$i "U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_nopp.so" || exit 1
done
