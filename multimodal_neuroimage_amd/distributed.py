"""Data-parallel runtime of the hot path: one process per GPU, batch sharded, gradients
averaged by a bucketed RCCL all-reduce overlapped with backward.

Mirrors what the reference's trainer does around the model (trainer.py:274-290: DDP with
find_unused_parameters; dataloaders.py:55-99: DistributedSampler(shuffle=True) + set_epoch),
re-shaped for MI355X:
  * backend "nccl" is RCCL on ROCm (xGMI between the GPUs of a node); "gloo" on CPU for tests;
  * DDP with static_graph=True instead of find_unused_parameters: SwinFusion never uses 18,702 of
    its parameters, and a static graph marks them once instead of
    traversing the autograd graph every step;
  * gradient_as_bucket_view=True: the gradients live inside the all-reduce buckets (no copy);
  * bucket_cap_mb: the 3D SwinFusion's 1.7 MB of gradients fit one bucket, so the whole exchange
    is a single ring all-reduce per step, issued as soon as backward reaches the first layers.
Rendezvous is always 127.0.0.1 (single node).
"""
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    local_rank: int = 0
    world: int = 1
    device: torch.device = torch.device("cpu")

    @property
    def enabled(self):
        return self.world > 1


def init_from_env(backend=None, use_cuda=None):
    """Read RANK / LOCAL_RANK / WORLD_SIZE (torch.distributed.run), bind the local GPU and init
    the process group when WORLD_SIZE > 1.  backend defaults to nccl (RCCL) on GPU, gloo on CPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if use_cuda is None:
        use_cuda = backend != "gloo"
    if use_cuda:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if use_cuda else "gloo")
        kw = dict(device_id=device) if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return DistEnv(rank=rank, local_rank=local, world=world, device=device)


def wrap_ddp(model, env, bucket_cap_mb=25):
    """DistributedDataParallel for the data-parallel path; identity for world == 1."""
    if not env.enabled:
        return model
    ids = [env.local_rank] if env.device.type == "cuda" else None
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids, broadcast_buffers=False,
                                                     gradient_as_bucket_view=True, static_graph=True,
                                                     bucket_cap_mb=bucket_cap_mb)


class ShardSampler:
    """DistributedSampler semantics (torch.utils.data.distributed.DistributedSampler, as the
    reference uses it at dataloaders.py:75): a per-epoch permutation seeded by (seed + epoch),
    padded to a multiple of world, rank r takes indices r, r + world, ...  drop_last drops the
    tail instead of padding."""

    def __init__(self, n, rank, world, shuffle=True, seed=0, drop_last=False):
        self.n, self.rank, self.world = n, rank, world
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and n % world:
            self.per_rank = n // world
        else:
            self.per_rank = -(-n // world)
        self.total = self.per_rank * world

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if self.drop_last:
            idx = idx[:self.total]
        else:
            pad = self.total - len(idx)
            idx += (idx * (pad // max(len(idx), 1) + 1))[:pad]
        return iter(idx[self.rank:self.total:self.world])

    def __len__(self):
        return self.per_rank


def max_over_ranks(value, env):
    """The slowest rank's wall time (bench contract: MAX over ranks)."""
    if not env.enabled:
        return float(value)
    t = torch.tensor([float(value)], device=env.device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(env):
    if env.enabled:
        dist.barrier()


def shutdown(env):
    if env.enabled and dist.is_initialized():
        dist.destroy_process_group()
