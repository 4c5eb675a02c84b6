"""Whole-step hipGraph capture for the native training step.

A training step of the 96^3 trunk issues ~440 libu3d launches (plus the loss, the bucketed all-reduce and
the SGD foreach kernels). Launched one by one from Python that is a host-bound stream; captured once into a
hipGraph (torch.cuda.CUDAGraph is hipGraph on ROCm) the whole step replays with one launch. Every kernel of
the step runs on every replay — nothing is cached — so replay does exactly the work of an eager step.

Requirements the native path meets: no host syncs (no .item()), every libu3d call is asynchronous on torch's
current stream (the capture stream during capture), scratch buffers are grow-only and reach their steady
size in the warm-up steps, parameter gradients are written into fresh tensors (set_to_none=True) that the
capture pool keeps at fixed addresses, or (data parallel, u3d.ddp) into bucket buffers allocated once. The kernel
forms of a data-parallel backward are chosen statically (ops.DDP_TOLERANT), never by polling a collective, so the
captured step is the step every eager run would take.

The reference has no train-step function (train_amos_atlas_final.py:209-399 runs it inline); this is the
additive helper Engine.graphed_train_step / bench.py use.
"""
import os

import torch


def _rccl_groups():
    """The initialised torch.distributed process groups whose backend is "nccl" (= RCCL on ROCm)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return []
    from torch.distributed import distributed_c10d as c10d
    out = []
    for pg in list(c10d._world.pg_map.keys()):
        try:
            if dist.get_backend(pg) == "nccl":
                out.append(pg)
        except (RuntimeError, ValueError):
            continue
    return out


def _check_event_cache():
    """ProcessGroupNCCL's event cache hands an event a captured collective recorded (a capture node) back to later
    works, and the watchdog's completion query of such an event aborts the process (hipErrorCapturedEvent; one abort
    on record, r05 `bench_fb1.log`). The cache is read when the process group is created, so the setting cannot be
    fixed here: fail loudly instead of aborting later in the watchdog. ``U3D_GRAPH_ALLOW_EVENT_CACHE=1`` skips the
    check (diagnostics only)."""
    if os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE") == "0" or os.environ.get("U3D_GRAPH_ALLOW_EVENT_CACHE") == "1":
        return
    raise RuntimeError("GraphedStep with an RCCL process group needs TORCH_NCCL_CUDA_EVENT_CACHE=0 in the environment "
                       "before the process group is created (bench.py and engine.py set it)")


class GraphedStep:
    """Capture ``step_fn() -> tensor`` once; ``__call__`` replays it and returns the captured output.

    ``static_inputs`` are the tensors the step reads; ``__call__(*new)`` copies ``new`` into them first
    (on the stream, inside the caller's timing) so each replay sees the new batch.
    """

    def __init__(self, step_fn, static_inputs=(), warmup=3, optimizer=None, capture_error_mode=None):
        """``capture_error_mode``: torch.cuda.graph's; default "thread_local" when torch.distributed is initialised
        (the process group's watchdog thread queries events of earlier collectives while this thread captures; the
        step's own all-reduces are captured as graph nodes on RCCL's stream, joined back by ``work.wait()``), else
        torch's "global"."""
        self.static_inputs = tuple(static_inputs)
        self.optimizer = optimizer
        rccl_groups = _rccl_groups()
        if capture_error_mode is None:
            import torch.distributed as dist
            capture_error_mode = "thread_local" if dist.is_available() and dist.is_initialized() else "global"
        if rccl_groups:
            _check_event_cache()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._zero()
                step_fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # Every warm-up collective has completed on the device; wait until each RCCL process group's watchdog has
        # also retired them (its work list empty), so no watchdog query of a pre-capture work is in flight when the
        # capture begins. A deterministic condition, not a delay: ProcessGroupNCCL::waitForPendingWorks.
        for pg in rccl_groups:
            pg._wait_for_pending_works()
        self.graph = torch.cuda.CUDAGraph()
        self._zero()
        try:
            with torch.cuda.graph(self.graph, capture_error_mode=capture_error_mode):
                self.out = step_fn()
        except Exception as e:
            # torch.cuda.graph leaves its capture stream current (and capturing) when capture_end raises (e.g. a gloo
            # collective's unjoined work): nothing on this device can run afterwards, so callers must not fall back to
            # eager in this process (bench.py decides eager up front for backends that cannot be captured)
            e.u3d_capture_started = True
            raise
        torch.cuda.synchronize()

    def _zero(self):
        if self.optimizer is not None:
            self.optimizer.zero_grad(set_to_none=True)

    def __call__(self, *new_inputs):
        for dst, src in zip(self.static_inputs, new_inputs):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        if hasattr(self.optimizer, "sync_lr"):
            self.optimizer.sync_lr()  # device-side lr of u3d.optim.SGD: LR schedule changes reach the replay
        self.graph.replay()
        return self.out
