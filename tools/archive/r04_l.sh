#!/bin/bash
# r04: shifted-fp32 brick epilogue statistics (parity + kbench vs the fp32 / fp64 forms), the default bench line
# (hipGraph at N=1, eager probe pass) next to an --eager line
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_l
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_pbrick.py tests/test_gpu_graph.py tests/test_gpu_gnfused_brick.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab46.so" "U3D_LIB=$L/libu3d_abcc.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py fwd48st fwd48st_nores fwd24st >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
timeout -k 10 300 python bench.py --no-cpu --no-infer > $O/bench_graph.log 2>&1 || { tail -20 $O/bench_graph.log; exit 1; }
grep '^{' $O/bench_graph.log | cut -c1-330
timeout -k 10 300 python bench.py --no-cpu --no-infer --eager > $O/bench_eager.log 2>&1 || { tail -20 $O/bench_eager.log; exit 1; }
grep '^{' $O/bench_eager.log | cut -c1-330
