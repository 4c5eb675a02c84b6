"""Benchmark: train voxels/s at 96^3 patch on 1..8 MI355X (BASELINE.json metric), one process per GPU.

Workload (BASELINE.json configs[1]; configs[2] at N=8): the reference's 16-organ trunk unet3D_baseline([1,2,2,2,2],
16, weight_std=True), batch 2x1x96^3 per GPU, bf16 activations (fp32 master weights, fp32 accumulation),
synthetic CT-like volumes, random-init weights. One step = forward + EDiceLoss_partial(16) (uce) + backward
(gradient all-reduce over RCCL inside the backward when N > 1) + SGD(momentum 0.9, wd 1e-4).

Prints ONE JSON line on rank 0. `roofline` is the dominant kernel (the 32->32 3^3 conv at 96^3, 50.9% of
forward FLOPs) timed with HIP events on the stream it is launched on; `cpu_baseline` times the oracle
(plain-PyTorch fp32 restatement) on this host's cores on the same 2x96^3 step (warm-up + median of 3).
`--gpus N` without WORLD_SIZE in the environment starts the N ranks itself (one process per GPU).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "multimodal-pl_amd"), REPO]

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
    p.add_argument("--print-rank-env", action="store_true", help=argparse.SUPPRESS)  # launcher test (no GPU)
    p.add_argument("--graph", action="store_true", help="replay the step as one captured hipGraph (~1%% faster at "
                   "N=1; the roofline kernel then falls back to a standalone timing: graph event nodes are not "
                   "timeable)")
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


def dominant_kernel_roofline(device, batch, patch, live=None, reps=20):
    """The 32->32 3^3 stride-1 conv (GN+ReLU prologue, residual epilogue) at patch^3, bf16. `live` = (avg ms,
    launches, voxels) from HIP events recorded around its launches inside the timed steps (on the stream it runs
    on); a standalone timing of the same launch is reported beside it (and used when `live` is None)."""
    from u3d import ops
    x = torch.randn((batch, patch, patch, patch, 32), device=device).to(torch.bfloat16)
    w = torch.randn(32, 32, 3, 3, 3, device=device)
    pf, _, _ = ops.wstd_fwd(w, torch.bfloat16, True, need_dgrad=False)
    st = ops.gn_stats(x, 16)
    ga = torch.ones(32, device=device)
    be = torch.zeros(32, device=device)
    for _ in range(3):  # the production launch: GroupNorm statistics accumulated in the epilogue
        y, _ = ops.conv_fwd_stats(x, pf, 32, 3, 1, (st, ga, be, 16), residual=x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        y, _ = ops.conv_fwd_stats(x, pf, 32, 3, 1, (st, ga, be, 16), residual=x)
    e1.record()
    torch.cuda.synchronize()
    ms_alone = e0.elapsed_time(e1) / reps
    flops = 2.0 * batch * patch ** 3 * 27 * 32 * 32
    ms, src = ms_alone, "standalone"
    if live is not None and live[2] == batch * patch ** 3:
        ms, src = live[0], f"HIP events, {live[1]} launches, {live[3]}"
    achieved = flops / (ms * 1e-3) / 1e12
    del y
    traffic, tsrc = pmc_traffic(batch, patch)
    kname = ops.CONV32_FN.replace("u3d_", "") + "_kernel"
    return {"kernel": "%s (conv 32->32 3^3 s1 @%d^3, GN+ReLU prologue, residual)" % (kname, patch),
            "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
            "traffic_source": tsrc, "algorithmic_bytes": 3 * batch * patch ** 3 * 32 * 2,
            "avg_launch_ms": round(ms, 4), "timing": src, "standalone_launch_ms": round(ms_alone, 4),
            "flop_per_launch": flops, "rocprof_check": timing_check(batch, patch, flops),
            "peak_measured": measured_peak(achieved)}


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


def pmc_traffic(batch, patch):
    """HBM bytes per launch of the dominant kernel from the newest committed rocprofv3 PMC summary
    (profiles/rNN_pmc_conv32_fwd.json, made by tools/pmc_traffic.py: 2*FETCH_SIZE + WRITE_SIZE, gfx950
    FETCH_SIZE correction). Only valid for the configuration it was measured on (2x96^3)."""
    f = newest_profile("pmc_conv32_fwd.json")
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


def timing_check(batch, patch, flops):
    """The newest committed cross-check of the live event timing against the rocprofv3 kernel trace of the same
    run (profiles/rNN_conv32_timing_check.json, tools/timing_check.py): reported beside `achieved`, with the
    roofline fraction the trace's in-step average gives. Only valid for the configuration it was measured on."""
    f = newest_profile("conv32_timing_check.json")
    if f is None or (batch, patch) != (2, 96):
        return None
    with open(f) as fh:
        c = json.load(fh)
    return {"file": os.path.relpath(f, REPO), "in_step_events_us": c["in_step_events_us"],
            "in_step_trace_us": c["in_step_trace_us"], "standalone_events_us": c["standalone_events_us"],
            "standalone_trace_us": c["standalone_trace_us"],
            "frac_at_trace_in_step": round(flops / (c["in_step_trace_us"] * 1e-6) / 1e12 / PEAK_BF16_TFLOPS, 4)}


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
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
        assert dist.get_world_size() == world

    import unet3D
    from loss_functions.loss_partial import EDiceLoss_partial
    from u3d.ddp import U3DDataParallel

    torch.manual_seed(0)
    model = unet3D.unet3D_baseline([1, 2, 2, 2, 2], num_classes=16, weight_std=True).to(device).train()
    net = U3DDataParallel(model) if world > 1 else model
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

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            logits, _, _ = net(x)
        loss = crit(logits, target, mask=[mask])
        loss.backward()
        opt.step()
        return loss

    graphed = None
    a.eager = not a.graph  # default: kernel-by-kernel launches (live HIP-event timing of the roofline kernel)
    from u3d import ops as _ops
    if not a.eager:
        from u3d.graph import GraphedStep
        try:
            _ops.PROBE = []  # the capture records event nodes around the dominant kernel; replays re-time them
            graphed = GraphedStep(step, (x, target, mask), warmup=3, optimizer=opt)
            probes = _ops.PROBE[-4:]
            _ops.PROBE = None
        except Exception as e:  # capture refused (e.g. a collective backend without graph support): run eager
            print(f"[bench] hipGraph capture failed ({type(e).__name__}: {e}); running eager", file=sys.stderr)
            torch.cuda.synchronize()
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
    if a.eager:
        _ops.PROBE = probes = []  # events around every dominant-kernel launch of the timed steps
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
    live = None
    try:  # dominant kernel timed live over the timed region (eager: every launch; graph: the last replay)
        # only the full-patch launches: the trunk also runs a 32->32 ring conv at half resolution, whose shorter
        # launch must not enter an average priced at the full-patch FLOPs
        full = a.batch * a.patch ** 3
        durs = [e0.elapsed_time(e1) for e0, e1, v in probes if v == full]
        if durs:
            live = (sum(durs) / len(durs), len(durs), full,
                    "every launch of the timed steps" if a.eager else "the last timed hipGraph replay")
    except Exception as e:  # noqa: BLE001 - event nodes not timeable on this runtime: fall back below
        print(f"[bench] live kernel timing unavailable ({e}); using the standalone measurement", file=sys.stderr)
    ms = dt / a.steps * 1e3
    vox = world * a.batch * a.patch ** 3 * a.steps / dt

    roof = None
    cpu = None
    if rank == 0 and not a.no_roofline:
        roof = dominant_kernel_roofline(device, a.batch, a.patch, live)
        step_gflop = STEP_GFLOP_PER_SAMPLE * a.batch * (a.patch / 96) ** 3
        roof["step_mfma_frac"] = round(step_gflop / (ms * 1e-3) / 1e3 / PEAK_BF16_TFLOPS, 4)
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
                       "backend": dist.get_backend() if world > 1 else None,
                       "world_size_seen": dist.get_world_size() if world > 1 else 1},
            "loss": round(loss_v, 6), "launch": "eager" if a.eager else "hipgraph",
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
