"""Benchmark: train voxels/s at 96^3 patch on 1..8 MI355X (BASELINE.json metric), one process per GPU.

Workload (BASELINE.json configs[1]; configs[2] at N=8): the reference's 16-organ trunk unet3D_baseline([1,2,2,2,2],
16, weight_std=True), batch 2x1x96^3 per GPU, bf16 activations (fp32 master weights, fp32 accumulation),
synthetic CT-like volumes, random-init weights. One step = forward + EDiceLoss_partial(16) (uce) + backward
(gradient all-reduce over RCCL inside the backward when N > 1) + SGD(momentum 0.9, wd 1e-4).

Prints ONE JSON line on rank 0. `roofline` is the ring kernel with the largest time per step among the full-patch
96^3 rings (the 32->32 3^3 convs: forward, data gradient with the fused GroupNorm-backward partials, and the stride-1
weight gradient), each launch timed with HIP events on the stream it runs on; the others are listed in
`roofline.rings`. `infer_cfg5` is BASELINE configs[4] (sliding-window inference of a 256x512x512 volume, 80 tiles,
bf16 and fp32). `cpu_baseline` times the oracle (plain-PyTorch fp32 restatement) on this host's cores on the same
2x96^3 step (warm-up + median of 3). `--gpus N` without WORLD_SIZE in the environment starts the N ranks itself (one
process per GPU); `--force-buckets` runs the N>1 gradient-bucket machinery on one GPU (RCCL at world size 1).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "multimodal-pl_amd"), REPO]

# RCCL collectives are captured into the step's hipGraph (N>1, --force-buckets). torch's process-group event cache
# can hand an event that was recorded inside the capture to the watchdog thread's completion query ("operation not
# permitted on an event last recorded in a capturing stream", seen once in r05): no cached events (set before the
# process group exists).
os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, no sparsity)
VOX96 = 96 ** 3
STEP_GFLOP_PER_SAMPLE = 1152.733  # fwd + dgrad + wgrad conv FLOPs per 96^3 sample (C=16)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=2, help="patches per GPU")
    p.add_argument("--patch", type=int, default=96)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--modality", default="ct", choices=["ct", "mixed"],
                   help="mixed = BASELINE configs[3]: per GPU one CT-normalised and one z-scored MRI-like patch "
                        "(MOTSDataset.py:171-185), the batch's mask[0] applied to both (loss_partial.py:87)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--no-infer", action="store_true", help="skip the configs[4] sliding-window inference leg")
    p.add_argument("--no-mixed", action="store_true", help="skip the configs[3] (CT + MRI batch) step leg at N=1")
    p.add_argument("--force-buckets", action="store_true",
                   help="N=1 only: RCCL (nccl backend) at world size 1 with U3DDataParallel(force_buckets=True), i.e. "
                        "the bucketed all-reduces launched from inside the backward and the collective-tolerant kernel "
                        "forms while they run (what N>1 pays for the overlap, measured on one GPU)")
    p.add_argument("--bucket-mb", type=float, default=25.0, help="gradient bucket cap (MB of fp32 gradients)")
    p.add_argument("--tail-mb", type=float, default=25.0, help="cap of the last bucket (launched at the backward's end)")
    p.add_argument("--print-rank-env", action="store_true", help=argparse.SUPPRESS)  # launcher test (no GPU)
    p.add_argument("--graph", action="store_true", help="replay the step as one captured hipGraph (the default, also at "
                   "N>1 and with --force-buckets; the ring kernels' live timing comes from an eager pass of the same "
                   "steps after the timed region)")
    p.add_argument("--eager", action="store_true", help="launch the step kernel by kernel from Python")
    return p.parse_args()


def synthetic(batch, patch, device, seed, modality="ct"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    hu = torch.rand((batch, 1, patch, patch, patch), generator=g) * 2000 - 1000
    x = hu.clamp(-325, 325) / 325                          # CT normalisation, MOTSDataset.py:171-182
    if modality == "mixed":                                # odd samples: MRI z-scored (MOTSDataset.py:183-185)
        mri = torch.rand((batch, 1, patch, patch, patch), generator=g) * 900
        mri = (mri - mri.mean(dim=(2, 3, 4), keepdim=True)) / mri.std(dim=(2, 3, 4), keepdim=True)
        x[1::2] = mri[1::2]
    x = x.to(device)
    lab = torch.randint(0, 16, (batch, 1, patch, patch, patch), generator=g).float().to(device)
    mask = (torch.rand(16, generator=g) < 0.6).long()
    mask[1] = 1
    return x, lab, mask


# the ring kernels the bench probes at the full patch, their committed-profile tag (profiles/rNN_pmc_<tag>.json) and the
# substring of their rocprofv3 kernel name + grid in profiles/rNN_kernel_summary.txt (tools/prof_summary.py)
RING_TAGS = {
    "wgrad_ring 32->32 GN": ("wgrad96", ("wgrad_ring_dma_kernel<true>', 1, '1', '256'",  # the 16 x 16-tile ring (LDS-DMA staging)
                                         "wgrad_ring_kernel<true, 16, 16>', 1, '1', '256'")),
    "conv32_ring dgrad +GN-bwd partials": ("dgrad96gn", "conv32_ring_kernel<true, true, false, 8, false, false>', 256"),
    "conv32_ring fwd GN +res +stats": ("fwd96", "conv32_ring_kernel<false, true, true, 12, false, false>', 256"),
    "conv32_ring fwd GN +stats": ("fwd96_nores", "conv32_ring_kernel<false, true, false, 16, false, false>', 256"),
}


def ring_groups(probes, full, steps):
    """Per (label) group of the full-patch ring launches recorded in the timed steps: launches, average event time,
    time per step, achieved TFLOP/s and the fraction of the dense bf16 peak."""
    groups = {}
    for e0, e1, label, flop, vox in probes:
        if vox == full:
            groups.setdefault(label, []).append((e0.elapsed_time(e1), flop))
    out = []
    for label, v in groups.items():
        avg = sum(t for t, _ in v) / len(v)
        flop = v[0][1]
        ach = flop / (avg * 1e-3) / 1e12
        out.append({"kernel": label, "launches_per_step": round(len(v) / steps, 2), "avg_launch_ms": round(avg, 4),
                    "ms_per_step": round(sum(t for t, _ in v) / steps, 4), "flop_per_launch": flop,
                    "achieved": round(ach, 2), "frac": round(ach / PEAK_BF16_TFLOPS, 4)})
    out.sort(key=lambda g: -g["ms_per_step"])
    return out


def standalone_ms(label, device, batch, patch, reps=20):
    """The same launch outside the step (random bf16 operands; hipGraph-free back-to-back launches): reported beside
    the live figure, and used for `achieved` when no live probe ran (e.g. --graph)."""
    from u3d import ops
    x = torch.randn((batch, patch, patch, patch, 32), device=device).to(torch.bfloat16)
    dy = torch.randn_like(x)
    w = torch.randn(32, 32, 3, 3, 3, device=device)
    pf, pd, _ = ops.wstd_fwd(w, torch.bfloat16, True)
    st = ops.gn_stats(x, 16)
    gn = (st, torch.ones(32, device=device), torch.zeros(32, device=device), 16)
    fns = {"wgrad_ring 32->32 GN": lambda: ops.conv_wgrad(dy, x, 3, 1, gn, brick="ring"),
           "conv32_ring dgrad +GN-bwd partials": lambda: ops.conv_dgrad_gn(dy, pd, 32, x, 3, 1, gn),
           "conv32_ring fwd GN +res +stats": lambda: ops.conv_fwd_stats(x, pf, 32, 3, 1, gn, residual=x),
           "conv32_ring fwd GN +stats": lambda: ops.conv_fwd_stats(x, pf, 32, 3, 1, gn)}
    fn = fns[label]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def algorithmic_bytes(label, batch, patch):
    """HBM bytes one launch of a full-patch 96^3-class ring must move (bf16 NDHWC tensors of batch x patch^3 x 32):
    * weight gradient: x and dy read + its fp32 split-K slabs written (splits x 27 x 32 x 32 x 4 B; 256 splits at
      2 x 96^3 = 28.3 MB) -> 254 MB at 2 x 96^3;
    * data gradient with the fused GroupNorm-backward partials: dy and x read, dA written -> 340 MB;
    * forward with GN prologue + residual: x and the residual read, y written -> 340 MB;
    * forward with GN prologue: x read, y written -> 226 MB."""
    t = batch * patch ** 3 * 32 * 2
    if label.startswith("wgrad_ring"):
        from u3d import _lib
        ns = _lib.query("u3d_conv_wgrad_ring_splits", batch, 32, patch, patch, patch, 32)
        return 2 * t + ns * 27 * 32 * 32 * 4
    if label == "conv32_ring fwd GN +stats":
        return 2 * t
    return 3 * t


def dominant_kernel_roofline(device, batch, patch, groups):
    """Roofline line of the ring kernel with the largest time per step (HIP events around each of its launches in the
    timed steps, on the stream it runs on); the other full-patch rings are carried beside it in `rings`."""
    if groups:
        dom = groups[0]
        label, ms, src = dom["kernel"], dom["avg_launch_ms"], "HIP events, every launch of the timed steps"
    else:
        label, ms, src = "wgrad_ring 32->32 GN", None, "standalone"
    ms_alone = standalone_ms(label, device, batch, patch)
    if ms is None:
        ms = ms_alone
    flops = 2.0 * batch * patch ** 3 * 27 * 32 * 32
    achieved = flops / (ms * 1e-3) / 1e12
    tag, krx = RING_TAGS.get(label, (None, None))
    traffic, tsrc = pmc_traffic(tag, batch, patch)
    return {"kernel": label, "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
            "traffic_unit": "bytes/launch", "traffic_source": tsrc,
            "algorithmic_bytes": algorithmic_bytes(label, batch, patch),
            "traffic_over_algorithmic": (round(traffic / algorithmic_bytes(label, batch, patch), 3)
                                         if traffic else None),
            "avg_launch_ms": round(ms, 4), "timing": src, "standalone_launch_ms": round(ms_alone, 4),
            "flop_per_launch": flops, "trace_check": trace_check(krx, flops) if (batch, patch) == (2, 96) else None,
            "peak_measured": measured_peak(achieved), "rings": groups}


def newest_profile(suffix):
    """The committed profile of the newest round: profiles/rNN_<suffix> with the highest NN; a plain `rNN_` file (the
    final tree of that round) wins over the round's intermediate `rNN<tag>_` files, whatever their names sort as."""
    import glob
    import re
    best = None
    for f in glob.glob(os.path.join(REPO, "profiles", "r*_" + suffix)):
        m = re.match(r"r(\d+)([a-z0-9]*)_" + re.escape(suffix) + "$", os.path.basename(f))
        if m:
            key = (int(m.group(1)), m.group(2) == "", m.group(2))
            if best is None or key > best[0]:
                best = (key, f)
    return None if best is None else best[1]


def pmc_traffic(tag, batch, patch):
    """HBM bytes per launch of a ring kernel from the newest committed rocprofv3 PMC summary
    (profiles/rNN_pmc_<tag>.json, made by tools/pmc_traffic.py: 2*FETCH_SIZE + WRITE_SIZE, gfx950 FETCH_SIZE
    correction). Only valid for the configuration it was measured on (2x96^3)."""
    f = newest_profile(f"pmc_{tag}.json") if tag else None
    if f is None or (batch, patch) != (2, 96):
        return None, None
    with open(f) as fh:
        return int(json.load(fh)["traffic_bytes"]), os.path.relpath(f, REPO)


def measured_peak(achieved):
    """The newest committed on-box calibration (profiles/rNN_peaks.json, tools/peak.hip: back-to-back bf16 MFMA on
    every CU at the clock held under load; HBM read/copy). `peak` stays the guide's dense figure; this is beside it."""
    f = newest_profile("peaks.json")
    if f is None:
        return None
    with open(f) as fh:
        c = json.load(fh)
    return {"file": os.path.relpath(f, REPO), "mfma_bf16_tflops": c["mfma_bf16_dense_tflops"],
            "hbm_read_gbs": c["hbm_read_gbs"], "frac_of_measured": round(achieved / c["mfma_bf16_dense_tflops"], 4)}


def trace_check(krx, flops):
    """The same kernel's in-step average from the newest committed rocprofv3 kernel-trace summary of the bench
    (profiles/rNN_kernel_summary.txt, tools/prof_summary.py) and the roofline fraction it gives: the live event
    figure must agree with it (events carry the markers' own cost, a few %)."""
    f = newest_profile("kernel_summary.txt")
    if f is None or krx is None:
        return None
    import re
    krxs = (krx,) if isinstance(krx, str) else krx
    with open(f) as fh:
        for line in fh:
            if any(k in line for k in krxs):
                m = re.search(r"avg=\s*([0-9.]+)us", line)
                if m:
                    us = float(m.group(1))
                    return {"file": os.path.relpath(f, REPO), "in_step_trace_us": us,
                            "frac_at_trace": round(flops / (us * 1e-6) / 1e12 / PEAK_BF16_TFLOPS, 4)}
    return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(batch, patch, reps=3):
    """Oracle (plain PyTorch fp32 CPU restatement, oracle/ref_cpu.py) timed on this host: SURVEY §8(d) procedure —
    the same workload as the GPU step (batch x 1 x patch^3, fwd + EDiceLoss_partial + bwd), one full-size warm-up,
    then the median of ``reps`` steps. Threads: every core of this process's affinity mask, capped by the
    OMP_NUM_THREADS share the box grants (16 per GPU on the pool; os.cpu_count() shows the whole machine there)."""
    import statistics
    from oracle import ref_cpu as O
    from oracle.weights_recipe import recipe_state_dict
    ncpu = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    torch.set_num_threads(max(1, min(ncpu, share) if share > 0 else ncpu))
    P = {k: torch.from_numpy(v).requires_grad_(True) for k, v in recipe_state_dict(O.state_shapes_baseline(16)).items()}
    x, lab, mask = synthetic(batch, patch, "cpu", 7)

    def step():
        for p in P.values():
            p.grad = None
        t0 = time.perf_counter()
        y = O.baseline_forward(P, x)
        loss = O.edice_partial(y, lab.squeeze(1), mask=[mask])
        loss.backward()
        return time.perf_counter() - t0

    warm = step()
    ts = [step() for _ in range(reps)]
    dt = statistics.median(ts)
    return {"value": round(batch * patch ** 3 / dt, 1), "unit": "voxels/s", "cores": torch.get_num_threads(),
            "cpu_model": _cpu_model(), "affinity_cores": ncpu, "kind": "port",
            "sample": f"{batch}x1x{patch}^3 training step (fwd+EDiceLoss_partial+bwd, fp32, oracle/ref_cpu.py): "
                      f"1 warm-up ({warm:.2f} s) + median of {reps} ({', '.join('%.2f' % t for t in ts)} s)"}


def infer_cfg5(device):
    """BASELINE configs[4] on this GPU: evaluate_amos.predict_sliding over one 1x1x256x512x512 volume, 64x192x192
    tiles, overlap 1/4 (80 tiles), the 16-organ trunk, forward only (bench_infer.measure: one warm-up volume, then one
    timed volume per dtype). fp32 is what the reference computes there (its --FP16 flag never casts:
    evaluate_amos.py:594-601); bf16 (fp32 accumulation) is the fast mode."""
    import bench_infer
    out = {"workload": "predict_sliding 1x1x256x512x512, tile 64x192x192, overlap 1/4, unet3D_baseline(16)",
           "data": "synthetic CT-like volume, random-init weights (resident on the device)"}
    for dt in ("bf16", "fp32"):
        out[dt] = bench_infer.measure(device, dt, reps=1)
    torch.cuda.empty_cache()
    return out


def mixed_leg(a, make_step, opt, device, rank):
    """BASELINE configs[3] per GPU at N=1: the same step on the multimodal batch (one CT-normalised patch, one z-scored
    MRI-like patch, MOTSDataset.py:171-185; the batch's mask[0] applied to both, loss_partial.py:87), same model and
    optimizer, its own captured hipGraph (or eager with --eager); warm-up + the same number of timed steps, timed like
    the main line (synchronize on both sides)."""
    bm = []
    for j in range(2):
        xb, lb, mb = synthetic(a.batch, a.patch, device, 2000 + 17 * j + rank, "mixed")
        bm.append((xb, lb.squeeze(1), mb.to(device)))
    xm, tm, mm = (t.clone() for t in bm[0])
    stepm = make_step(xm, tm, mm)
    if a.eager:
        def run(i):
            for dst, src in zip((xm, tm, mm), bm[i % 2]):
                dst.copy_(src, non_blocking=True)
            return stepm()
    else:
        from u3d.graph import GraphedStep
        g = GraphedStep(stepm, (xm, tm, mm), warmup=3, optimizer=opt)
        def run(i):
            return g(*bm[i % 2])
    for i in range(a.warmup):
        run(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = run(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = dt / a.steps * 1e3
    return {"workload": "configs[3] per GPU: same step, batch = 1 CT-normalised + 1 z-scored MRI-like 96^3 patch",
            "ms_per_step": round(ms, 3), "value": round(a.batch * a.patch ** 3 * a.steps / dt, 1), "unit": "voxels/s",
            "launch": "eager" if a.eager else "hipgraph", "loss": round(float(loss), 6)}


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N child ranks (RANK / LOCAL_RANK / WORLD_SIZE, rendezvous on
    127.0.0.1) before this process touches the GPU, pass their output through, exit with the worst status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def capturable():
    """Whether the step's collectives can be captured into a hipGraph: RCCL (backend "nccl") can, gloo cannot."""
    return not dist.is_initialized() or dist.get_backend() == "nccl"


def launch_mode(a, world):
    """'graph' (hipGraph replay of the whole step, its bucketed RCCL all-reduces included at N>1 / --force-buckets)
    unless --eager; a refused capture falls back to eager and says so in the line (`launch`, `graph_error`)."""
    return "eager" if a.eager else "graph"


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))
    if a.print_rank_env:
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}))
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # U3D_BENCH_BACKEND=gloo with U3D_BENCH_SHARE_GPU=1: rehearse the N>1 path on a one-GPU box (every rank on device
    # local % count, gloo collectives on device tensors: the bucketed all-reduce, the ranks' agreement on graph vs eager
    # — gloo collectives cannot be captured — and the max-over-ranks timing). Not a scaling measurement.
    backend = os.environ.get("U3D_BENCH_BACKEND", "nccl")
    if os.environ.get("U3D_BENCH_SHARE_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group(backend, init_method="env://")
        assert dist.get_world_size() == world
    elif a.force_buckets:
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)

    import unet3D
    from loss_functions.loss_partial import EDiceLoss_partial
    from u3d.ddp import U3DDataParallel

    torch.manual_seed(0)
    model = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(device).train()
    net = (U3DDataParallel(model, force_buckets=a.force_buckets, bucket_mb=a.bucket_mb, tail_mb=a.tail_mb)
           if (world > 1 or a.force_buckets) else model)
    from u3d.optim import SGD  # drop-in for torch.optim.SGD: one fused launch per 48 tensors
    opt = SGD(model.parameters(), lr=5e-4, momentum=0.9, weight_decay=1e-4)
    crit = EDiceLoss_partial(16)
    # two resident synthetic batches; each step consumes the other one (copied into the step's input buffers)
    batches = []
    for j in range(2):
        xb, lb, mb = synthetic(a.batch, a.patch, device, 1000 + 17 * j + rank, a.modality)
        batches.append((xb, lb.squeeze(1), mb.to(device)))
    x, target, mask = (t.clone() for t in batches[0])
    amp = a.dtype == "bf16"

    def make_step(x, target, mask):
        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                logits, _, _ = net(x)
            loss = crit(logits, target, mask=[mask])
            loss.backward()
            opt.step()
            return loss
        return step

    step = make_step(x, target, mask)

    graphed = None
    graph_error = None
    # the step replays as one hipGraph (the Python host launching ~180 library calls per step was measured slower than
    # the GPU runs them: eager 6.03-6.19 vs graph 5.98-6.01 ms/step, gpurun_out/r04_k); at N>1 / --force-buckets the
    # bucketed RCCL all-reduces are captured with it (their kernel forms are static: ops.DDP_TOLERANT)
    a.eager = launch_mode(a, world) == "eager" or not capturable()
    from u3d import ops as _ops
    if not a.eager:
        from u3d.graph import GraphedStep
        try:
            graphed = GraphedStep(step, (x, target, mask), warmup=3, optimizer=opt)
        except Exception as e:  # refused before the capture began (e.g. the event-cache check): run eager
            if getattr(e, "u3d_capture_started", False):
                raise  # the device's capture stream is left capturing: no eager fallback in this process
            graph_error = f"{type(e).__name__}: {e}"[:300]
            print(f"[bench] hipGraph capture failed ({graph_error}); running eager", file=sys.stderr)
            torch.cuda.synchronize()
            a.eager = True
        if dist.is_initialized():
            # every rank replays or every rank runs eager: a rank-local fallback would leave the ranks issuing
            # different collective sequences (captured vs eager all-reduces) and mis-pair or hang them
            ok = torch.tensor([0 if a.eager else 1], dtype=torch.int32, device=device)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and not a.eager:
                graph_error = "hipGraph capture failed on another rank; every rank runs eager"
                print(f"[bench] {graph_error}", file=sys.stderr)
                graphed = None
                a.eager = True
    if a.eager:
        def run(i):
            x.copy_(batches[i % 2][0], non_blocking=True)
            target.copy_(batches[i % 2][1], non_blocking=True)
            mask.copy_(batches[i % 2][2], non_blocking=True)
            return step()
    else:
        def run(i):
            return graphed(*batches[i % 2])

    for i in range(a.warmup):
        run(i)
    probes = []
    probe_pass = None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = run(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    loss_v = float(loss)
    _ops.PROBE = None
    if not a.no_roofline:  # (every rank: the step may hold collectives)
        # the ring kernels' live timing (HIP events around every launch) comes from an eager pass of the same step
        # right after the timed region: graph replay has no per-launch events, and the events' host cost (~0.4 ms per
        # eager step, r04) stays out of the timed steps
        _ops.PROBE = probes
        for i in range(a.steps):
            x.copy_(batches[i % 2][0], non_blocking=True)
            target.copy_(batches[i % 2][1], non_blocking=True)
            mask.copy_(batches[i % 2][2], non_blocking=True)
            step()
        torch.cuda.synchronize()
        _ops.PROBE = None
        probe_pass = f"eager pass of {a.steps} steps after the timed region"
    groups = []
    try:  # the full-patch ring launches only (the trunk also runs ring kernels at 48^3 and below)
        groups = ring_groups(probes, a.batch * a.patch ** 3, a.steps)
    except Exception as e:  # noqa: BLE001 - event timing unavailable: fall back to the standalone launch
        print(f"[bench] live kernel timing unavailable ({e}); using the standalone measurement", file=sys.stderr)
    ms = dt / a.steps * 1e3
    vox = world * a.batch * a.patch ** 3 * a.steps / dt

    mixed = None
    if world == 1 and a.modality == "ct" and not a.no_mixed:
        mixed = mixed_leg(a, make_step, opt, device, rank)
    roof = None
    cpu = None
    infer = None
    if rank == 0 and not a.no_roofline:
        roof = dominant_kernel_roofline(device, a.batch, a.patch, groups)
        if probe_pass:
            roof["probe_pass"] = probe_pass
            if groups:
                roof["timing"] = "HIP events, every launch of the " + probe_pass
        step_gflop = STEP_GFLOP_PER_SAMPLE * a.batch * (a.patch / 96) ** 3
        roof["step_mfma_frac"] = round(step_gflop / (ms * 1e-3) / 1e3 / PEAK_BF16_TFLOPS, 4)
    if rank == 0 and world == 1 and not a.no_infer:
        infer = infer_cfg5(device)
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(a.batch, a.patch)
    if rank == 0:
        out = {
            "metric": "train voxels/sec at 96^3 patch, 1/2/4/8 MI355X; fwd+bwd step ms",
            "value": round(vox, 1), "unit": "voxels/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": a.dtype, "data": "synthetic (CT-normalised random volumes, random labels, random-init weights)",
            "config": {"workload": "unet3D_baseline([1,2,2,2,2],16,weight_std) fwd+EDiceLoss_partial+bwd+SGD",
                       "model": "unet3D_baseline-16", "global_batch": world * a.batch, "seq_len": a.patch ** 3,
                       "patch": [a.patch] * 3, "parallelism": f"dp{world}",
                       "backend": dist.get_backend() if dist.is_initialized() else None,
                       "world_size_seen": dist.get_world_size() if dist.is_initialized() else 1,
                       "force_buckets": bool(a.force_buckets)},
            "loss": round(loss_v, 6), "launch": "eager" if a.eager else "hipgraph", "graph_error": graph_error,
            "ddp_tolerant_forms": bool(_ops.DDP_TOLERANT[0]),
            "roofline": roof, "cpu_baseline": cpu, "infer_cfg5": infer, "mixed_cfg3": mixed,
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
