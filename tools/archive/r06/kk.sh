#!/bin/bash
# round 6: conv1 weight gradient with 4-plane bricks (A, the tree) vs 2 (libu3d_bd2) and 8 (libu3d_bd8): its tests,
# kbench 3 rounds, then a step A/B of A vs bd2, 3 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06kk; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  -k "stem" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
U3D_LIB=$R/multimodal-pl_amd/u3d/libu3d_bd8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_bf16.py -k "stem_wgrad" > $O/tests8.log 2>&1 || { tail -30 $O/tests8.log; exit 1; }
tail -1 $O/tests8.log
for i in 1 2 3; do for L in "" bd2 bd8; do
  echo "== ${L:-bd4}" >> $O/kb.log
  U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/libu3d_$L.so} timeout -k 10 120 python tools/kbench.py stemw96 >> $O/kb.log 2>&1 || exit 1
done; done
grep -A1 "==" $O/kb.log | grep -v "^--"
for i in 1 2 3; do for L in "" bd2; do
  ms=$(U3D_LIB=${L:+$R/multimodal-pl_amd/u3d/libu3d_$L.so} timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "${L:-bd4} $ms" | tee -a $O/ab.log
done; done
