#!/bin/bash
# round 6: GroupNorm coefficient loads issued together (gn_coef8): GPU suite, kernel A/B, step A/B vs libu3d_ab.so
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06y; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/kab.sh r06y 2 wgrad6 wgrad12 wgrad24 wgrad96 fwd96 dgrad96gn wgrad1_96 head96 || exit 1
for i in 1 2 3; do for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
  ms=$(U3D_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "${L:+B}${L:-A} $ms" | tee -a $O/ab.log
done; done
