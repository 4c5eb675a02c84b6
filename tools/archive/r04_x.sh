#!/bin/bash
# r04: 32 partial pairs per round in the GN-backward last-block combine (in-tree) vs 8 (HEAD, libu3d_ab.so); parity first
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_x
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_gnfused.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$R/multimodal-pl_amd/u3d
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so"; do
    echo "== $v" >> $O/kab.log
    env $v timeout -k 10 120 python tools/kbench.py gnbwd2s96 gnbwd2s48 gnbwd2s24 gnbwd2s12 gnbwd248 gnbwd224 gnbwd212 gnbwd96 gnbwd48 gnbwd24 gnbwd12 >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/kab.log
for i in 1 2; do
  for v in "U3D_X=0" "U3D_LIB=$L/libu3d_ab.so"; do
    ms=$(env $v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 40 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "$v $ms" | tee -a $O/ab.log
  done
done
