#!/bin/bash
# round 6: step A/B of the tree (A) against the MFMA-stem commit d837e80 (B: libu3d_ab.so), 4 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06ii; mkdir -p $O; cd $R
for i in 1 2 3 4; do for L in "" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"; do
  ms=$(U3D_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-roofline --steps 30 --warmup 5 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
  echo "${L:+B}${L:-A} $ms" | tee -a $O/ab.log
done; done
