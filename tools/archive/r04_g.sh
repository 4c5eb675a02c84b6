#!/bin/bash
# r04: brick GN-backward epilogue with the x loads issued under the last tap plane: parity, kernel A/B (in-tree vs
# libu3d_ab.so = previous commit: dgrad48gn / dgrad24gn / the forward bricks), step A/B (U3D_GN_BWD_FUSED_BRICK=0/1),
# then the implicit-GEMM depth sweep (tools/r04_f.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_g
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_gnfused_brick.py tests/test_gpu_pbrick.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py gnb48f gnb48s gnb24f gnb24s dgrad48gn dgrad24gn fwd48 fwd24 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
for i in 1 2 3; do
  for v in 1 0; do
    ms=$(U3D_GN_BWD_FUSED_BRICK=$v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "fused_brick=$v $ms" | tee -a $O/ab.log
  done
done
bash tools/r04_f.sh
