import torch
dev = torch.device("cuda:0")
def t_(fn, reps=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
for M, N, K in [(3456, 256, 6912), (432, 320, 8640), (27648, 128, 3456), (6912, 256, 3456), (221184, 64, 1728)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    bt = b.t().contiguous()
    us = t_(lambda: a @ b)
    us2 = t_(lambda: a @ bt.t())
    print(M, N, K, f"{us:.1f}us {2*M*N*K/us/1e6:.0f} TF | NT {us2:.1f}us {2*M*N*K/us2/1e6:.0f} TF", flush=True)
