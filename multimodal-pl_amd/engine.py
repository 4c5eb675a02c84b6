"""Drop-in for the reference engine.py (Engine runtime facade, engine.py:10-76).

Same constructor, attributes and methods (.args, .distributed, .local_rank, .world_size, .devices,
data_parallel, get_train_loader, get_test_loader, all_reduce_tensor, context manager, injected -d/-c
flags). Unlike the CPU stub in the reference snapshot, this one is a real multi-process runtime: one process
per GPU launched by torchrun (RANK / LOCAL_RANK / WORLD_SIZE env), RCCL ("nccl" backend on ROCm) over xGMI,
and data_parallel() returns the native bucketed-all-reduce wrapper (u3d.ddp). On a CPU-only host with
WORLD_SIZE > 1 it uses gloo (tests).
"""
import argparse
import os

import torch
import torch.distributed as dist

from utils import all_reduce_tensor as _all_reduce_tensor
from utils import extant_file


class Engine(object):
    def __init__(self, custom_parser=None):
        self.devices = None
        self.distributed = False
        if custom_parser is None:
            self.parser = argparse.ArgumentParser()
        else:
            assert isinstance(custom_parser, argparse.ArgumentParser)
            self.parser = custom_parser
        self.inject_default_parser()
        self.args = self.parser.parse_args()  # as the reference (engine.py:22): unknown flags are an error
        self.continue_state_object = self.args.continue_fpath

        self.world_size = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", getattr(self.args, "local_rank", 0) or 0))
        self.rank = int(os.environ.get("RANK", self.local_rank))
        self.distributed = self.world_size > 1
        use_cuda = torch.cuda.is_available()
        if self.distributed:
            if use_cuda:
                torch.cuda.set_device(self.local_rank % max(1, torch.cuda.device_count()))
            if not dist.is_initialized():
                # no cached process-group events: the step may be captured into a hipGraph with its all-reduces
                # (u3d.graph.GraphedStep), and a cached event recorded inside the capture must not reach the watchdog
                os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
                dist.init_process_group(backend="nccl" if use_cuda else "gloo", init_method="env://")
            self.devices = list(range(self.world_size))
        else:
            self.devices = [0]

    @property
    def device(self):
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    def data_parallel(self, model):
        from u3d.ddp import U3DDataParallel
        return U3DDataParallel(model)

    def graphed_train_step(self, step_fn, static_inputs=(), optimizer=None, warmup=3):
        """Additive helper (the reference runs its step inline, train_amos_atlas_final.py:209-399): capture
        ``step_fn`` (forward, loss, backward, optimizer step on the tensors in ``static_inputs``) once as a hipGraph,
        data-parallel all-reduces included; calling the result with new batches replays it (u3d.graph.GraphedStep)."""
        from u3d.graph import GraphedStep
        return GraphedStep(step_fn, static_inputs, warmup=warmup, optimizer=optimizer)

    def get_train_loader(self, train_dataset, collate_fn=None):
        train_sampler = None
        is_shuffle = True
        batch_size = self.args.batch_size
        if self.distributed:
            train_sampler = torch.utils.data.distributed.DistributedSampler(train_dataset)
            batch_size = max(1, self.args.batch_size // self.world_size)
            is_shuffle = False
        train_loader = torch.utils.data.DataLoader(train_dataset, batch_size=batch_size,
                                                   num_workers=getattr(self.args, "num_workers", 0), drop_last=False,
                                                   shuffle=is_shuffle, pin_memory=torch.cuda.is_available(),
                                                   sampler=train_sampler, collate_fn=collate_fn)
        return train_loader, train_sampler

    def get_test_loader(self, test_dataset):
        test_sampler = None
        if self.distributed:
            test_sampler = torch.utils.data.distributed.DistributedSampler(test_dataset, shuffle=False)
        test_loader = torch.utils.data.DataLoader(test_dataset, batch_size=1,
                                                  num_workers=getattr(self.args, "num_workers", 0), drop_last=False,
                                                  shuffle=False, pin_memory=torch.cuda.is_available(),
                                                  sampler=test_sampler)
        return test_loader, test_sampler

    def all_reduce_tensor(self, tensor, norm=True):
        if self.distributed:
            return _all_reduce_tensor(tensor, world_size=self.world_size, norm=norm)
        return torch.mean(tensor)

    # ---------------------------------------------------------------------------------------- additive
    def train_step(self, model, optimizer, images, labels, sup_mask):
        """One pre-train step as train_amos_atlas_final.py:258-378 runs it for the trunk: forward, partial
        Dice+BCE (get_loss pre-train branch), backward (gradient all-reduce inside), SGD step."""
        from loss_functions.losses import get_loss
        optimizer.zero_grad(set_to_none=True)
        out = model(images, labels)
        preds = out[0] if isinstance(out, (tuple, list)) else out
        loss, _ = get_loss(preds, 0, [], labels, [sup_mask])
        loss.backward()
        optimizer.step()
        return loss

    def eval_step(self, model, images, labels, num_class):
        from evaluate_amos import get_dice
        with torch.no_grad():
            preds = model(images)
            preds = preds[0] if isinstance(preds, (tuple, list)) else preds
            return get_dice(preds, labels, 1, num_class=num_class)

    def inject_default_parser(self):
        p = self.parser
        p.add_argument("-d", "--devices", default="", help="set data parallel training")
        p.add_argument("-c", "--continue", type=extant_file, metavar="FILE", dest="continue_fpath",
                       help="continue from one certain checkpoint")

    def __enter__(self):
        return self

    def __exit__(self, type, value, tb):
        if type is not None:
            print("A exception occurred during Engine initialization, give up running process")
            return False
