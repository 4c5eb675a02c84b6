#!/bin/bash
# r04: GroupNorm-backward partials in the persistent brick data gradient (48^3 / 24^3): parity, kernel A/B
# (data gradient + whole GN backward, fused vs separate), step A/B (U3D_GN_BWD_FUSED_BRICK=0/1 alternating)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_e
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_gnfused_brick.py tests/test_gpu_gnfused.py tests/test_gpu_pbrick.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 120 python tools/kbench.py gnb48f gnb48s gnb24f gnb24s dgrad48 dgrad48gn dgrad24 dgrad24gn >> $O/kab.log 2>&1 || { tail $O/kab.log; exit 1; }
done
grep -v amdgpu.ids $O/kab.log
for i in 1 2 3; do
  for v in 1 0; do
    ms=$(U3D_GN_BWD_FUSED_BRICK=$v timeout -k 10 200 python bench.py --no-cpu --no-roofline --no-infer --steps 30 2>>$O/ab.err | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])") || exit 1
    echo "fused_brick=$v $ms" | tee -a $O/ab.log
  done
done
