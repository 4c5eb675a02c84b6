"""CPU-side checks: the C-ABI library loads and exports every symbol include/u3d.h declares, the drop-in
modules keep the reference's names / signatures / state_dict keys, the host logic (class weights, engine
flags, DDP bucketing over gloo with world_size 2) behaves like the reference. No compute calls here."""
import os
import re
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, golden


def _header_symbols():
    src = open(os.path.join(REPO, "include", "u3d.h")).read()
    return sorted(set(re.findall(r"\b(u3d_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from u3d import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libu3d.so not built")
    h = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(h, s), s
        assert s in _lib.exported_symbols(), f"{s} missing from the ctypes signature table"
    assert h.u3d_abi_version() == 1


def test_library_has_no_undefined_internal_symbols():
    """Every u3d:: function the library calls is defined in it (a shared object links with undefined symbols, which
    would only fail at load time on the GPU box)."""
    import shutil
    import subprocess
    from u3d import _lib
    if not os.path.exists(_lib.LIB_PATH) or shutil.which("nm") is None:
        pytest.skip("libu3d.so or nm missing")
    out = subprocess.run(["nm", "-DC", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    bad = [ln for ln in out.splitlines() if "u3d::" in ln or " u3d_" in ln]
    assert not bad, bad


def test_workspace_size_constants_match_the_library():
    from u3d import _lib, ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libu3d.so not built")
    assert _lib.query("u3d_stem_fwd_ws_bytes") == ops.STEM_WS_BYTES


def test_header_compiles_as_c():
    import subprocess
    r = subprocess.run(["gcc", "-fsyntax-only", "-x", "c", os.path.join(REPO, "include", "u3d.h")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_state_dict_keys_match_reference():
    import unet3D
    for name, ctor in [("g3_baseline16_16.npz", lambda: unet3D.unet3D_baseline([1, 2, 2, 2, 2], 16, True)),
                       ("g1_unet3d_dyn_32.npz", lambda: unet3D.UNet3D(2, True)),
                       ("g2_unet3d_g_32.npz",
                        lambda: unet3D.unet3D_g([1] * 5, num_classes=2, weight_std=True, init_filter=24, in_channel=2))]:
        m = ctor()
        assert [k for k, _ in m.named_parameters()] == list(golden(name)["gnames"])
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], 16, True)
    assert m.layer1[0].conv1.weight.shape == (64, 32, 3, 3, 3)
    assert sum(p.numel() for p in m.parameters()) == 17286512  # 16-class trunk


def test_unet3d_param_count():
    import unet3D
    assert sum(p.numel() for p in unet3D.UNet3D(2, True).parameters()) == 17329528  # SURVEY A8 probe


def test_reference_names_exported():
    import evaluate_amos
    import unet3D
    from loss_functions import loss_partial, losses
    for n in ["unet3D_with_feam3", "get_style_discriminator_output", "norm_style_discriminator_output",
              "deep_style_discriminator_output", "unet3D_with_deepsup", "unet3D_g", "UNet3D", "unet3D_with_eam",
              "unet3D_with_eam_baseline", "unet3D_with_feam2", "unet3D_baseline", "Conv3d", "conv3x3x3",
              "NoBottleneck"]:
        assert hasattr(unet3D, n), n
    for n in ["DiceLoss", "EDiceLoss_partial", "EDiceLoss_full", "EDiceLoss_full2"]:
        assert hasattr(loss_partial, n)
    assert hasattr(losses, "get_loss")
    for n in ["dice_score", "spec_score", "senc_score", "get_dice", "get_dice2", "predict_sliding"]:
        assert hasattr(evaluate_amos, n)


def test_cpu_forward_raises_not_falls_back():
    import unet3D
    from u3d import U3DError
    m = unet3D.unet3D_baseline([1, 2, 2, 2, 2], 16, True)
    with pytest.raises(U3DError):
        m(torch.zeros(1, 1, 16, 16, 16))


def test_class_weights_quirks():
    from u3d.loss import class_weights
    w = class_weights([torch.tensor([0, 1, 1, 0, 1]), torch.tensor([1, 1, 1, 1, 1])], 4, "cpu")
    assert w.tolist() == [0.0, 1.0, 1.0, 0.0]  # mask[0] only, truncated to C
    assert class_weights(None, 3, "cpu").tolist() == [1.0, 1.0, 1.0]
    with pytest.raises(IndexError):
        class_weights([torch.ones(15)], 16, "cpu")


def test_dice_score_helpers_match_oracle():
    from evaluate_amos import dice_score, senc_score, spec_score
    rng = np.random.default_rng(0)
    p = torch.from_numpy(rng.random((2, 1000)) > 0.5)
    t = torch.from_numpy(rng.random((2, 1000)) > 0.7)
    num = (p & t).sum(1).double()
    np.testing.assert_allclose(float(dice_score(p, t)), (2 * num / (p.sum(1) + t.sum(1) + 1)).mean().item(), rtol=1e-6)
    np.testing.assert_allclose(float(senc_score(p, t)), (num / (t.sum(1) + 1)).mean().item(), rtol=1e-6)
    np.testing.assert_allclose(float(spec_score(p, t)), (num / (p.sum(1) + 1)).mean().item(), rtol=1e-6)


def test_engine_flags_and_single_process():
    import argparse
    import engine
    p = argparse.ArgumentParser()
    p.add_argument("--batch_size", type=int, default=2)
    import sys
    old = sys.argv
    sys.argv = ["x", "-d", "0"]
    try:
        with engine.Engine(custom_parser=p) as e:
            assert e.args.devices == "0" and e.world_size == 1 and not e.distributed
            assert float(e.all_reduce_tensor(torch.tensor([1.0, 3.0]))) == 2.0
            m = torch.nn.Linear(2, 2)
            w = e.data_parallel(m)
            assert w.module is m
        sys.argv = ["x", "--no-such-flag"]
        with pytest.raises(SystemExit):  # parse_args, as the reference: unknown flags are rejected
            engine.Engine(custom_parser=argparse.ArgumentParser())
    finally:
        sys.argv = old


def test_lr_poly():
    import utils
    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0)
    lr = utils.adjust_learning_rate(opt, 10, 0.01, 100, 0.9)
    assert abs(lr - 0.01 * (0.9 ** 0.9)) < 1e-12 and opt.param_groups[0]["lr"] == lr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from u3d.ddp import GradBucketer, U3DDataParallel
    torch.manual_seed(rank)
    params = [(f"p{i}", torch.nn.Parameter(torch.randn(n))) for i, n in enumerate([5, 300, 7, 1000, 3])]
    b = GradBucketer(params, bucket_mb=0.002)  # ~524 floats per bucket -> several buckets
    assert len(b.buckets) >= 3
    b.begin()
    for n, p in reversed(params):
        if n == "p2":
            continue  # never produced -> zero-filled, still reduced
        b.out(n).fill_(float(rank + 1) * (1 + int(n[1:])))
        b.done(n)
    b.finish()
    vals = {n: b.view(n).clone() for n, _ in params}
    m = torch.nn.Linear(3, 3)
    torch.manual_seed(100 + rank)
    m.reset_parameters()
    U3DDataParallel(m)
    q.put((rank, {k: v.tolist() for k, v in vals.items()}, m.weight.detach().clone().tolist(), True))
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(target, world, timeout=120):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=timeout) for _ in procs), key=lambda o: o[0])
    for p in procs:
        p.join(timeout=timeout)
        assert p.exitcode == 0
    return out


def _check_bucketer(world):
    out = _run_ranks(_ddp_worker, world)
    for rank, vals, w, _ in out:
        for n, v in vals.items():
            i = int(n[1:])
            expect = 0.0 if n == "p2" else (world + 1) / 2 * (1 + i)  # mean over ranks of (rank+1)*(1+i)
            assert np.allclose(v, expect), (n, v[:3], expect)
    for o in out[1:]:
        assert np.allclose(out[0][2], o[2])  # init broadcast: identical weights on every rank


def test_ddp_bucketer_gloo_world2():
    _check_bucketer(2)


def test_ddp_bucketer_gloo_world8():
    """BASELINE configs[2]'s rank count (8 x 2 patches = global batch 16) rehearsed on the CPU: the same buckets, the
    AVG over 8 ranks and the initial broadcast, through gloo (the RCCL path itself never ran beyond world 1 here)."""
    _check_bucketer(8)


def _used_flags_worker(rank, world, port, q):
    """DDP's unused-parameter semantics through the bucket flags: p2 is produced on rank 0 only (both ranks get the
    averaged slice), p4 on no rank (.grad stays None on both: no weight decay / momentum on it, as on one GPU)."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from u3d.ddp import GradBucketer
    params = [(f"p{i}", torch.nn.Parameter(torch.randn(n))) for i, n in enumerate([5, 300, 7, 1000, 3])]
    b = GradBucketer(params, bucket_mb=0.002)
    out = []
    for step in range(2):  # the second step reads the flags again (eager: no cached answer)
        for _, p in params:
            p.grad = None
        b.begin()
        for n, p in reversed(params):
            if n == "p4" or (n == "p2" and rank != 0):
                continue
            b.out(n).fill_(float(rank + 1) * (1 + int(n[1:])))
            b.done(n)
        b.finish()
        out.append({n: (None if p.grad is None else p.grad.tolist()) for n, p in params})
    q.put((rank, out, sorted(b.assigned)))
    dist.barrier()
    dist.destroy_process_group()


def _check_used_flags(world):
    out = _run_ranks(_used_flags_worker, world)
    for rank, steps, assigned in out:
        assert assigned == (["p0", "p1", "p2", "p3"] if rank == 0 else ["p0", "p1", "p3"])
        for grads in steps:
            assert grads["p4"] is None, (rank, "a parameter no rank produced must keep grad None")
            assert np.allclose(grads["p2"], 3.0 / world), (rank, grads["p2"][:3])  # rank 0's (0+1)*3 over the ranks
            for i in (0, 1, 3):
                assert np.allclose(grads[f"p{i}"], (world + 1) / 2 * (1 + i)), (rank, i)


def test_ddp_used_flags_gloo_world2():
    _check_used_flags(2)


def test_ddp_used_flags_gloo_world8():
    """p2 produced on rank 0 of 8 only, p4 on none: the used flags ride the last bucket's AVG at configs[2]'s rank
    count."""
    _check_used_flags(8)


def _fallback_worker(rank, world, port, q):
    """Plain torch autograd parameters (no native tape) under U3DDataParallel: every gradient reaches the
    post-accumulate hook and is averaged; equals one process on the concatenated batch."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from u3d.ddp import U3DDataParallel
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 2))
    net = U3DDataParallel(m)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 6, generator=g)
    net(x[2 * rank:2 * rank + 2]).square().mean().backward()
    grads = {k: p.grad.tolist() for k, p in m.named_parameters()}
    q.put((rank, grads, sorted(net.fallback_names)))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_fallback_hook_averages_non_native_grads_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 2))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 6, generator=g)
    (0.5 * (m(x[:2]).square().mean() + m(x[2:]).square().mean())).backward()
    for rank, grads, fallback in out:
        assert fallback == sorted(k for k, _ in m.named_parameters())
        for k, p in m.named_parameters():
            assert np.allclose(grads[k], p.grad.numpy(), rtol=1e-6, atol=1e-7), (rank, k)



def _fallback_mismatch_worker(rank, world, port, q):
    """Rank 1's backward reaches a parameter rank 0's does not: both ranks must raise, not hang or mis-pair."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from u3d.ddp import U3DDataParallel
    torch.manual_seed(0)
    m = torch.nn.ModuleList([torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)])
    net = U3DDataParallel(m)
    x = torch.randn(2, 4)
    y = net.module[0](x) if rank == 0 else net.module[1](net.module[0](x))
    try:
        y.sum().backward()
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, "raised" if "different sets" in str(e) else repr(e)))
    dist.destroy_process_group()


def test_ddp_fallback_mismatch_fails_loudly_gloo_world2():
    """ranks whose backward reaches different non-native parameters raise instead of hanging."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_mismatch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert out == [(0, "raised"), (1, "raised")], out

class _NativeScale(torch.autograd.Function):
    """Stands in for a native tape (u3d.trunk._TrunkFn) in CPU tests: its parameter's gradient is written straight into
    the DDP bucket and the bucketer's begin()/finish() run around it; ``boom`` makes its backward raise."""

    @staticmethod
    def forward(ctx, x, w, boom):
        from u3d.ddp import current_sink
        ctx.sink, ctx.boom = current_sink(), boom
        ctx.save_for_backward(x)
        if ctx.sink is not None:
            ctx.sink.begin()
        return x * w

    @staticmethod
    def backward(ctx, g):
        if ctx.boom:
            raise RuntimeError("boom")
        x, = ctx.saved_tensors
        gw = (g * x).sum(0)
        out = ctx.sink.out("w") if ctx.sink is not None else None
        if out is not None:
            out.copy_(gw)
            ctx.sink.done("w")
            ctx.sink.finish()
            gw = ctx.sink.returned(["w"], [out])[0]  # None: finish() set .grad to the averaged bucket view
        return g * 0 + g, gw, None


class _NativeModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.linspace(0.5, 1.5, 4))
        self.lin = torch.nn.Linear(4, 3)
        self.boom = False

    def forward(self, x, extra=True):
        y = _NativeScale.apply(x, self.w, self.boom)
        return self.lin(y) if extra else y


def _empty_set_worker(rank, world, port, q):
    """Rank 0 reaches no non-native parameter at all (only the native one); rank 1 reaches the Linear: both ranks
    must raise (rank 0 joins the consistency all-gather from the native finish()), none may hang."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from u3d.ddp import U3DDataParallel
    torch.manual_seed(0)
    net = U3DDataParallel(_NativeModel())
    try:
        net(torch.randn(2, 4), extra=rank == 1).sum().backward()
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, "raised" if "different sets" in str(e) else repr(e)))
    dist.destroy_process_group()


def test_ddp_fallback_mismatch_with_an_empty_rank_fails_loudly_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_set_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert out == [(0, "raised"), (1, "raised")], out


def _raise_then_step_worker(rank, world, port, q):
    """A backward that raises after the fallback hooks fired: the next step must still average both the
    native bucket gradient and the fallback (Linear) gradients."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from u3d.ddp import U3DDataParallel
    torch.manual_seed(0)
    m = _NativeModel()
    net = U3DDataParallel(m)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 4, generator=g)
    m.boom = True
    try:
        net(x[2 * rank:2 * rank + 2]).square().sum().backward()
        first = "no error"
    except RuntimeError as e:
        first = str(e)
    m.boom = False
    for p in m.parameters():
        p.grad = None
    net(x[2 * rank:2 * rank + 2]).square().sum().backward()
    q.put((rank, first, {k: p.grad.tolist() for k, p in m.named_parameters()}, sorted(net.fallback_names)))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_step_after_a_raised_backward_still_averages_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_raise_then_step_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    m = _NativeModel()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 4, generator=g)
    (0.5 * (m(x[:2]).square().sum() + m(x[2:]).square().sum())).backward()
    for rank, first, grads, fallback in out:
        assert "boom" in first, first
        assert fallback == ["lin.bias", "lin.weight"], fallback
        for k, p in m.named_parameters():
            assert np.allclose(grads[k], p.grad.numpy(), rtol=1e-6, atol=1e-7), (rank, k, grads[k], p.grad)


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus N` (the driver's SCALE command shape, no torchrun) starts N ranks itself, each with
    its own RANK / LOCAL_RANK / WORLD_SIZE and a 127.0.0.1 rendezvous, before any GPU call."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--print-rank-env"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = sorted((json.loads(s) for s in r.stdout.strip().splitlines()), key=lambda d: d["RANK"])
    assert [(d["RANK"], d["LOCAL_RANK"], d["WORLD_SIZE"], d["MASTER_ADDR"]) for d in lines] == \
        [(str(i), str(i), "3", "127.0.0.1") for i in range(3)]


def test_bench_launch_mode_defaults():
    """bench.py times hipGraph replays by default, also where the step holds its bucketed all-reduces (N>1,
    --force-buckets: the kernel forms are static, ops.DDP_TOLERANT); --eager launches kernel by kernel."""
    import argparse
    import sys
    sys.path.insert(0, REPO)
    import bench

    def ns(**k):
        d = dict(eager=False, graph=False, force_buckets=False)
        d.update(k)
        return argparse.Namespace(**d)
    assert bench.launch_mode(ns(), 1) == "graph"
    assert bench.launch_mode(ns(eager=True), 1) == "eager"
    assert bench.launch_mode(ns(force_buckets=True), 1) == "graph"
    assert bench.launch_mode(ns(), 8) == "graph"
    assert bench.launch_mode(ns(eager=True), 8) == "eager"


# ------------------------------------------------------------- f1: sliding-window tiles sharded over ranks
def test_tile_plan_matches_reference_tiling_and_shards_partition_it():
    from evaluate_amos import shard_tiles, tile_plan
    plan = tile_plan((1, 1, 256, 512, 512), (64, 192, 192))
    assert len(plan) == 80                                   # 5 x 4 x 4 tiles
    assert plan[0] == (0, 64, 0, 192, 0, 192) and plan[-1] == (192, 256, 320, 512, 320, 512)
    for world in (1, 2, 3, 8):
        shards = [shard_tiles(plan, r, world) for r in range(world)]
        assert sorted(t for s in shards for t in s) == sorted(plan)
        assert max(map(len, shards)) - min(map(len, shards)) <= 1
    small = tile_plan((1, 1, 40, 50, 30), (16, 24, 24))      # ragged: last tiles clamped back into the volume
    assert all(d2 - d1 == 16 and y2 - y1 == 24 and x2 - x1 == 24 for d1, d2, y1, y2, x1, x2 in small)


def _tile_pred(img):
    """Deterministic stand-in network for the sharding test: per-class affine maps of the tile."""
    return np.concatenate([img * (k + 1) - k for k in range(3)], axis=1)


def _window_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from evaluate_amos import shard_tiles, tile_plan
    from oracle.ref_cpu import gaussian_map
    rng = np.random.default_rng(5)
    image = rng.standard_normal((1, 1, 40, 50, 30))
    tile = (16, 24, 24)
    g = gaussian_map(tile).astype(np.float64)
    full = torch.zeros((1, 3, 40, 50, 30), dtype=torch.float64)
    count = torch.zeros((1, 3, 40, 50, 30), dtype=torch.float64)
    for d1, d2, y1, y2, x1, x2 in shard_tiles(tile_plan(image.shape, tile), rank, world):
        pred = _tile_pred(image[:, :, d1:d2, y1:y2, x1:x2])
        full[:, :, d1:d2, y1:y2, x1:x2] += torch.from_numpy(pred * g)
        count[:, :, d1:d2, y1:y2, x1:x2] += torch.from_numpy(g)
    dist.all_reduce(full)     # the product path's two all-reduces (evaluate_amos.predict_sliding)
    dist.all_reduce(count)
    q.put((rank, (full / count).numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_sliding_window_sharded_gloo_world2_matches_oracle():
    from oracle.ref_cpu import predict_sliding
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_window_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=60) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    image = np.random.default_rng(5).standard_normal((1, 1, 40, 50, 30))
    ref = predict_sliding(_tile_pred, image, (16, 24, 24), 3)
    for _, got in out:
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)


def test_driver_helpers_match_reference_fixture():
    """utils.mask_aug and the discriminator losses on the driver's import line (train_amos_atlas_final.py:34-35)
    against the reference's own outputs (G12)."""
    from loss_functions.losses import SmoothCrossEntropyLoss, bce_loss
    from utils import mask_aug
    g = golden("g12_driver_helpers.npz")
    assert np.array_equal(mask_aug(g["aug_in"], 2), g["aug_out"])
    assert np.array_equal(mask_aug(g["aug_in"], 3), g["aug_out3"])
    assert mask_aug(g["aug_in"], 1) is g["aug_in"] or np.array_equal(mask_aug(g["aug_in"], 1), g["aug_in"])
    with pytest.raises(TypeError):       # np.zeros(dtype=torch.float32), as in the reference
        mask_aug(torch.zeros(1, 1, 2, 2, 2), 2)
    t = torch.from_numpy(g["sce_t"])
    for tag, kw in (("plain", {}), ("smooth", dict(smoothing=0.2)), ("sum", dict(reduction="sum"))):
        x = torch.from_numpy(g["sce_x"]).requires_grad_(True)
        v = SmoothCrossEntropyLoss(**kw)(x, t)
        v.backward()
        np.testing.assert_allclose(float(v), float(g[f"sce_{tag}_value"]), rtol=1e-6)
        np.testing.assert_allclose(x.grad.numpy(), g[f"sce_{tag}_grad"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(float(bce_loss(torch.from_numpy(g["sce_x"]), 1)), float(g["bce1_value"]), rtol=1e-6)


def test_driver_import_line_resolves():
    """Every name train_amos_atlas_final.py imports from the drop-in modules exists (:19, :27, :29, :34, :35)."""
    import engine
    import evaluate_amos
    import unet3D
    import utils
    from loss_functions import losses
    for mod, names in ((unet3D, ["unet3D_with_feam3", "get_style_discriminator_output", "norm_style_discriminator_output",
                                 "deep_style_discriminator_output", "unet3D_with_deepsup", "unet3D_g"]),
                       (evaluate_amos, ["predict_sliding", "get_dice", "get_dice2"]), (engine, ["Engine"]),
                       (utils, ["adjust_learning_rate", "mask_aug", "seedfix"]),
                       (losses, ["get_loss_refine", "get_loss", "SmoothCrossEntropyLoss", "bce_loss"])):
        for n in names:
            assert hasattr(mod, n), (mod.__name__, n)


def test_no_kernel_spills_to_scratch():
    """no kernel of the shipped library spills VGPRs or uses a private (scratch) segment — read from
    the AMDGPU metadata notes of the gfx950 code objects inside libu3d.so (tools/kernel_resources.py)."""
    import shutil
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import kernel_resources as KR
    lib = os.path.join(REPO, "multimodal-pl_amd", "u3d", "libu3d.so")
    if not os.path.exists(lib) or not os.path.exists(os.path.join(KR.LLVM, "llvm-readelf")):
        pytest.skip("library or llvm tools not present")
    ks = KR.kernels(lib)
    assert len(ks) > 100, len(ks)
    bad = {k: v for k, v in ks.items() if v[".vgpr_spill_count"] or v[".private_segment_fixed_size"]}
    assert not bad, "kernels with VGPR spills / scratch: " + ", ".join(
        f"{n} ({v['.vgpr_spill_count']} spills, {v['.private_segment_fixed_size']} B)" for n, v in
        zip(KR.demangle(list(bad)), bad.values()))


def test_trace_step_marker_names_a_shipped_conv1_kernel():
    """tools/trace_steps.py splits a kernel trace into steps at the conv1 kernel (profile fidelity):
    its marker must match a kernel the library ships (round 6 moved conv1 to stem1_mfma_kernel; a stale marker made
    the steady-state summaries silently empty)."""
    import re
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import kernel_resources as KR
    import trace_steps
    lib = os.path.join(REPO, "multimodal-pl_amd", "u3d", "libu3d.so")
    if not os.path.exists(lib) or not os.path.exists(os.path.join(KR.LLVM, "llvm-readelf")):
        pytest.skip("library or llvm tools not present")
    names = KR.demangle(list(KR.kernels(lib)))
    hits = [nm for nm in names if re.search(trace_steps.MARKER, nm)]
    assert any("stem1_mfma_kernel" in nm for nm in hits), hits


def test_stride2_dgrad_beyond_2gib_routes_to_the_64bit_kernel(monkeypatch):
    """the stride-2 data-gradient kernel addresses dy with 32-bit buffer offsets, so a dy of 2 GiB or more
    must route to the 64-bit implicit-GEMM data gradient instead of failing with EINVAL (routing only: meta tensors,
    the library calls recorded, nothing launched)."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    from u3d import ops
    calls = []
    monkeypatch.setattr(ops, "call", lambda name, *a: calls.append(name))
    monkeypatch.setattr(ops, "_stream", lambda: 0)
    monkeypatch.setattr(ops.WS, "get", lambda *a, **k: torch.empty(256, dtype=torch.uint8, device="meta"))
    wpk = torch.empty((27, 32, 64), dtype=torch.bfloat16, device="meta")
    big = torch.empty((2, 48, 512, 512, 64), dtype=torch.bfloat16, device="meta")  # 3 GiB
    assert big.numel() * 2 >= (1 << 31)
    ops.conv_dgrad(big, wpk, 32, (2, 96, 1024, 1024), 3, 2)
    ops.conv_dgrad(torch.empty((2, 24, 64, 64, 64), dtype=torch.bfloat16, device="meta"), wpk, 32, (2, 48, 128, 128),
                   3, 2)
    assert calls == ["u3d_conv_dgrad", "u3d_conv_dgrad_s2"], calls


def test_dgrad_gn_routing_brick_levels(monkeypatch):
    """conv_dgrad_gn takes the persistent brick with the GN-backward partials in its epilogue
    (u3d_convg_brick_dgrad_gn) where conv_dgrad runs that brick and the volume is small (24^3 level); at 48^3 and for
    the 32-channel ring shapes it declines or takes the ring's own fused form (routing only: meta tensors, calls
    recorded, nothing launched)."""
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-pl_amd")]
    from u3d import ops
    calls = []
    monkeypatch.setattr(ops, "call", lambda name, *a: calls.append(name))
    monkeypatch.setattr(ops, "_stream", lambda: 0)
    monkeypatch.setattr(ops, "query", lambda name, *a: 54 if name == "u3d_convg_brick_gn_nparts" else 64)

    def gn(c):
        return (torch.empty((2, 16, 2), device="meta"), torch.empty(c, device="meta"), torch.empty(c, device="meta"), 16)

    def run(s, c):
        x = torch.empty((2, s, s, s, c), dtype=torch.bfloat16, device="meta")
        dy = torch.empty((2, s, s, s, c), dtype=torch.bfloat16, device="meta")
        wpk = torch.empty((27, c, c), dtype=torch.bfloat16, device="meta")
        return ops.conv_dgrad_gn(dy, wpk, c, x, 3, 1, gn(c))

    r = run(24, 128)
    assert r is not None and r[1].shape == (2, 54, 128, 2) and calls == ["u3d_convg_brick_dgrad_gn"], calls
    calls.clear()
    assert run(48, 64) is None and calls == []          # 48^3: the separate partial pass measured faster
    assert run(12, 256) is None and calls == []         # small-volume kernel level: no fused form
    monkeypatch.setattr(ops, "GN_BWD_FUSED_BRICK", False)
    assert run(24, 128) is None and calls == []


def test_compact_stride2_gn_backward_limits():
    """the paired GroupNorm backward reading the compact stride-2 1^3 data gradient (u3d_gn_bwd2_s2) needs
    < 2^24 voxels per sample and a compact operand < 2 GiB; outside them the trunk takes conv_dgrad + gn_bwd2."""
    from u3d import ops
    assert ops.s2_compact_ok((2, 96, 96, 96), 32, 2)
    assert ops.s2_compact_ok((2, 192, 192, 192), 32, 2)              # 7.1M voxels per sample
    assert not ops.s2_compact_ok((1, 256, 256, 256), 32, 2)          # 2^24 voxels per sample
    assert not ops.s2_compact_ok((16, 240, 240, 240), 64, 2)         # compact operand 2.8 GB
