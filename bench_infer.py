"""Inference benchmark for BASELINE.json configs[4]: evaluate_amos.predict_sliding over one 1x256x512x512 volume,
tile 64x192x192, overlap 1/4 (80 tiles, evaluate_amos.py:211-221), the 16-organ unet3D_baseline trunk, forward
only, bf16 activations (the config names fp16; the native path computes bf16 with fp32 accumulation), device
Gaussian accumulation. Prints one JSON line: volume voxels/s, per-tile ms and the conv-stack MFMA fraction
(1025.7 GFLOP per tile forward).

Multi-GPU (one process per GPU, `python -m torch.distributed.run --nproc-per-node N bench_infer.py`): the tiles are
sharded round-robin over the ranks (predict_sliding(..., group=WORLD), two RCCL all-reduces at the end); the time
is the max over ranks between barriers; the value is whole-volume voxels/s."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "multimodal-pl_amd"), REPO]

import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0
PEAK_F32_MFMA_TFLOPS = 157.3  # f32-input MFMA = the f32 vector peak (MI355X_MICROARCH.md, Matrix cores table)
GFLOP_PER_TILE = 1025.7


def tile_count(volume, tile, tta=False):
    """Tiles predict_sliding visits (evaluate_amos.py:215-221: overlap 1/4, ceil strides)."""
    import math
    D, H, W = volume
    sHW, sD = math.ceil(tile[1] * 0.75), math.ceil(tile[0] * 0.75)
    return ((math.ceil((D - tile[0]) / sD) + 1) * (math.ceil((H - tile[1]) / sHW) + 1)
            * (math.ceil((W - tile[2]) / sHW) + 1)) * (8 if tta else 1)


def measure(dev, dtype="bf16", reps=2, volume=(256, 512, 512), tile=(64, 192, 192), classes=16, tta=False, group=None):
    """Seconds per volume of predict_sliding (min over ``reps`` timed runs after one warm-up) and the derived rates.
    Forward only; the volume is resident on the device before the timed region (no host transfer inside it)."""
    import unet3D
    import evaluate_amos as E
    dist = None
    if group is not None:
        import torch.distributed as dist
    torch.manual_seed(0)  # random-init weights (the module's own init; nothing from oracle/)
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=classes, weight_std=True)
    m = m.to(dev).eval()
    m.compute_dtype = torch.bfloat16 if dtype == "bf16" else torch.float32
    g = torch.Generator(device="cpu").manual_seed(0)
    D, H, W = volume
    vol = ((torch.rand((1, 1, D, H, W), generator=g) * 2000 - 1000).clamp(-325, 325) / 325).to(dev)
    with torch.no_grad():
        out = E.predict_sliding(None, [m], vol, list(tile), classes, None, tta=tta, group=group)  # warm-up
        torch.cuda.synchronize()
        del out
        ts = []
        for _ in range(reps):
            if group is not None:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = E.predict_sliding(None, [m], vol, list(tile), classes, None, tta=tta, group=group)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if group is not None:
                tt = torch.tensor([dt], device=dev)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                dt = float(tt)
            ts.append(dt)
            del out
    tiles = tile_count(volume, tile, tta)
    t = min(ts)
    gflop = GFLOP_PER_TILE * tiles * (tile[0] * tile[1] * tile[2]) / (64 * 192 * 192)
    return {"dtype": dtype, "s_per_volume": round(t, 4), "voxels_per_s": round(D * H * W / t, 1), "tiles": tiles,
            "ms_per_tile": round(1e3 * t / tiles, 3), "conv_tflops": round(gflop / t / 1e3, 2),
            # against the peak of the dtype the convs compute in (fp32: the f32 MFMA / vector peak)
            "mfma_frac": round(gflop / t / 1e3 / (PEAK_F32_MFMA_TFLOPS if dtype == "fp32" else PEAK_BF16_TFLOPS), 4),
            "mfma_peak_tflops": PEAK_F32_MFMA_TFLOPS if dtype == "fp32" else PEAK_BF16_TFLOPS,
            "runs_s": [round(x, 4) for x in ts]}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--volume", type=int, nargs=3, default=[256, 512, 512])
    p.add_argument("--tile", type=int, nargs=3, default=[64, 192, 192])
    p.add_argument("--classes", type=int, default=16)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--tta", action="store_true")
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    group = None
    if world > 1:
        import torch.distributed as dist
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
        group = dist.group.WORLD
    else:
        dev = torch.device("cuda:0")
    r = measure(dev, a.dtype, a.reps, tuple(a.volume), tuple(a.tile), a.classes, a.tta, group)
    if group is not None and dist.get_rank() != 0:
        dist.destroy_process_group()
        return
    print(json.dumps({"metric": "sliding-window inference voxels/sec (configs[4])", "value": r["voxels_per_s"],
                      "n_gpus": world, "unit": "voxels/s", **r,
                      "data": "synthetic CT-like volume, random-init weights",
                      "config": {"workload": "unet3D_baseline(16) predict_sliding", "volume": a.volume,
                                 "tile": a.tile, "tta": a.tta}}))
    if group is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
