"""oracle/ — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

A plain-PyTorch fp32 CPU restatement of the reference's 3D U-Net segmentation path
(TThuraya/multimodal-PL: unet3D.py, loss_functions/loss_partial.py, evaluate_amos.py), pinned against
golden vectors produced by importing the reference itself (tests/golden/gen_golden.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import anything from here, and only
as the checker / CPU baseline. The product path (multimodal-pl_amd/) never imports it and has no CPU fallback.
"""
