#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
python -c "import torch; p=torch.cuda.get_device_properties(0); print('CUs', p.multi_processor_count, p.name)"
for w in 256 248 240 224 192 128; do
  for v in 0 1; do
    echo "== WGS $w V2 $v"; U3D_RING_WGS=$w U3D_RING_V2=$v timeout -k 10 60 python tools/kbench.py fwd96_plain dgrad96 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
