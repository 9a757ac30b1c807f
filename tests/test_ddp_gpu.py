"""The data-parallel path with the HIP kernels in the loop: two ranks (gloo over CUDA tensors, both
on cuda:0 — the single-GPU box cannot host two RCCL ranks) wrap SwinFusion with
distributed.wrap_ddp (static graph, gradient bucket views) and step on different pairs; the
DDP-averaged gradients must equal the mean of the two ranks' plain local gradients."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    sys.path.insert(0, os.path.dirname(HERE))
    import recipe
    import torch.distributed as dist
    from multimodal_neuroimage_amd import distributed as D
    from multimodal_neuroimage_amd import model as M
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK="0",
                      WORLD_SIZE=str(world), HSA_ENABLE_IPC_MODE_LEGACY="0")
    env = D.init_from_env(backend="gloo", use_cuda=True)
    kw = dict(fine_tune_task="binary_classification", size_of_model="large", swin_embed_dim=12, drop_rate=0.0,
              attn_drop_rate=0.0, mlp_ratio=4.0, drop_path_rate=0.0, intermediate_vec=84, patch_size=7,
              window_size=6, no_init_weights=True)
    local = M.SwinFusion(**kw)
    recipe.fill_params(local)
    local = local.to(env.device)
    ddp_model = M.SwinFusion(**kw)
    ddp_model.load_state_dict(local.state_dict())
    for mdl in (local, ddp_model):   # the Swin-V2 head's hard-coded drop_path 0.1 is RNG: off
        for mod in mdl.modules():
            if hasattr(mod, "drop_prob"):
                mod.drop_prob = 0.0
    ddp = D.wrap_ddp(ddp_model.to(env.device), env)
    A = torch.from_numpy(recipe.randn(7000 + rank, (1, 84, 84))).to(env.device)
    B = torch.from_numpy(recipe.randn(7100 + rank, (1, 84, 84))).to(env.device)
    y = torch.tensor([[float(rank)]], device=env.device)
    lossf = torch.nn.functional.binary_cross_entropy_with_logits
    for _ in range(2):   # static graph: same graph every step
        ddp.zero_grad(set_to_none=True)
        lossf(ddp(A, B)["binary_classification"], y).backward()
    local.zero_grad(set_to_none=True)
    lossf(local(A, B)["binary_classification"], y).backward()
    mine = {k: p.grad.detach().clone() for k, p in local.named_parameters() if p.grad is not None}
    avg = {}
    for k, g in mine.items():
        t = g.clone()
        dist.all_reduce(t)
        avg[k] = t / world
    worst, where = 0.0, ""
    for k, p in ddp.module.named_parameters():
        if k in avg:
            ref = avg[k]
            # per tensor, relative to that tensor's own gradient scale (every kernel's weight
            # gradient is a fixed-order reduction, so the two paths differ only by the all-reduce's
            # rounding; all-zero gradients of parameters the loss does not reach compare absolutely)
            e = float((p.grad - ref).abs().max() / max(float(ref.abs().max()), 1e-12))
            if e > worst:
                worst, where = e, f"{k}: ddp max {float(p.grad.abs().max()):.3e} ref max {float(ref.abs().max()):.3e}"
    out[rank] = (worst, where)
    D.shutdown(env)


def test_ddp_two_ranks_average_hip_gradients(device):
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _port(), out), nprocs=world, join=True)
    for r in range(world):
        worst, where = out[r]
        assert worst < 1e-4, f"rank {r}: max rel diff {worst:.2e} at {where}"
