"""The N>1 data-parallel path on CPU: two gloo ranks (world_size 2, 127.0.0.1) run the same
DDP wrapping, sharding and max-over-ranks timing reduction that bench.py uses over RCCL on GPUs
(multimodal_neuroimage_amd/distributed.py).  The model here is a small CPU stand-in with the
block's token-op structure (LayerNorm -> Linear -> GELU -> Linear); the HIP kernels themselves
need a GPU and are covered by the -m gpu tests."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

from multimodal_neuroimage_amd import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.norm = nn.LayerNorm(12)
        self.fc1 = nn.Linear(12, 48)
        self.fc2 = nn.Linear(48, 12)
        self.unused = nn.Linear(12, 12)     # like SwinFusion's never-used conv_first*_B (Q5)
        self.head = nn.Linear(12, 1)

    def forward(self, x):
        x = x + self.fc2(nn.functional.gelu(self.fc1(self.norm(x))))
        return self.head(x.mean(dim=1))


def _batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(3, 10, 12, generator=g), torch.randint(0, 2, (3, 1), generator=g).float()


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    env = D.init_from_env(backend="gloo")
    assert env.enabled and env.rank == rank and env.world == world
    torch.manual_seed(0)
    model = D.wrap_ddp(_Block(), env)
    x, y = _batch(rank)
    for step in range(2):      # static_graph needs the same graph every step
        model.zero_grad(set_to_none=True)
        nn.functional.binary_cross_entropy_with_logits(model(x), y).backward()
    grads = {k: p.grad.clone() for k, p in model.module.named_parameters() if p.grad is not None}
    t = D.max_over_ranks(1.0 + rank, env)
    s = D.ShardSampler(10, rank, world, shuffle=True, seed=3)
    s.set_epoch(1)
    out[rank] = dict(grads=grads, tmax=t, shard=list(s))
    D.barrier(env)
    D.shutdown(env)


def test_ddp_gloo_world2_averages_gradients_and_reduces_time():
    world, port = 2, _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    # reference: the mean of the per-rank gradients, computed in one process
    torch.manual_seed(0)
    ref_model = _Block()
    per_rank = []
    for r in range(world):
        ref_model.zero_grad(set_to_none=True)
        x, y = _batch(r)
        nn.functional.binary_cross_entropy_with_logits(ref_model(x), y).backward()
        per_rank.append({k: p.grad.clone() for k, p in ref_model.named_parameters() if p.grad is not None})
    for k in per_rank[0]:
        mean = (per_rank[0][k] + per_rank[1][k]) / 2
        for r in range(world):
            torch.testing.assert_close(out[r]["grads"][k], mean, rtol=1e-5, atol=1e-6)
    assert all("unused" not in k for k in out[0]["grads"])
    assert out[0]["tmax"] == out[1]["tmax"] == 2.0
    # shards are disjoint and cover every sample
    assert sorted(out[0]["shard"] + out[1]["shard"]) == list(range(10))


@pytest.mark.parametrize("n,world,drop_last", [(10, 2, False), (11, 4, False), (11, 4, True), (3, 8, False)])
def test_shard_sampler_matches_distributed_sampler(n, world, drop_last):
    from torch.utils.data.distributed import DistributedSampler
    data = list(range(n))
    for rank in range(world):
        ours = D.ShardSampler(n, rank, world, shuffle=True, seed=7, drop_last=drop_last)
        ref = DistributedSampler(data, num_replicas=world, rank=rank, shuffle=True, seed=7, drop_last=drop_last)
        for epoch in (0, 3):
            ours.set_epoch(epoch)
            ref.set_epoch(epoch)
            assert list(ours) == list(ref)
            assert len(ours) == len(ref)


def test_single_process_env_is_a_no_op():
    env = D.DistEnv()
    m = nn.Linear(2, 2)
    assert D.wrap_ddp(m, env) is m
    assert D.max_over_ranks(3.5, env) == 3.5


def _writer_worker(rank, world, port, out):
    from multimodal_neuroimage_amd.trainer import Writer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    env = D.init_from_env(backend="gloo")
    w = Writer(["train", "val"], 0.5, env=env, fine_tune_task="binary_classification")
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(12, generator=g)
    truth = (torch.arange(12) % 3 == 0).float()
    mine = [i for i in range(12) if i % world == rank]          # each rank validates its shard
    w.record("val", torch.tensor(mine), logits[mine], truth[mine])
    for k in range(2):
        w.write_losses({"binary_classification": torch.tensor(0.5 + rank + k), "total": torch.tensor(0.5 + rank + k)},
                       "val")
    w.loss_summary(lr=0)
    w.accuracy_summary(mid_epoch=False)
    out[rank] = dict(metrics=w.current_metrics, loss=w.total_val_loss_history[-1])
    D.shutdown(env)


def test_writer_gathers_predictions_over_ranks():
    """Validation metrics are computed over ALL ranks' subjects (the reference computes them per
    rank on its shard), and the loss summary is the mean over ranks."""
    from multimodal_neuroimage_amd.metrics import classification_metrics
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_writer_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(12, generator=g)
    truth = (torch.arange(12) % 3 == 0).float()
    ref = classification_metrics(truth.tolist(), torch.sigmoid(logits).tolist(), "val", 0.5)
    for r in range(world):
        assert out[r]["metrics"] == pytest.approx(ref, rel=1e-6)
        assert out[r]["loss"] == pytest.approx(1.5)     # mean of rank 0 (0.5, 1.5) and rank 1 (1.5, 2.5)
