#!/bin/bash
# r04: stride-2 data gradient as 4-wave workgroups, two per CU (libu3d_s2nt256.so, -DU3D_S2_NT=256) vs the 8-wave
# one-per-CU kernel (in-tree): parity under the variant, kernel A/B, step A/B (alternating x3)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_h
mkdir -p $O
cd $R
L=$R/multimodal-pl_amd/u3d
U3D_LIB=$L/libu3d_s2nt256.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -k "dgrad" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_s2nt256.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py dgrad_s2_96 dgrad_s2_48 dgrad_s2_24 dgrad_s2_12 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
for i in 1 2 3; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_s2nt256.so"; do
    ms=$(env $v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "$v $ms" | tee -a $O/ab.log
  done
done
