"""Standalone timing of the token ops at the C3 row count (4 x 96^3 tokens) vs torch:
LayerNorm fwd/bwd (C=12) and the Linear weight gradients of the SwinFusion block."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF  # noqa: E402

dev = torch.device("cuda:0")
rows = 4 * 96 ** 3
reps = 10


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {}
x = torch.randn(rows, 12, device=dev, requires_grad=True)
ln = torch.nn.LayerNorm(12).to(dev)
g = torch.randn(rows, 12, device=dev)
res["ln_fwdbwd_hip_ms"] = timeit(lambda: torch.autograd.backward(MF.layer_norm(x, ln), g))
res["ln_fwdbwd_torch_ms"] = timeit(lambda: torch.autograd.backward(ln(x), g))
for N, K in [(36, 12), (12, 12), (48, 12), (12, 48)]:
    xi = torch.randn(rows, K, device=dev)
    w = torch.randn(N, K, device=dev, requires_grad=True)
    b = torch.randn(N, device=dev, requires_grad=True)
    gy = torch.randn(rows, N, device=dev)
    y = MF.linear(xi, w, b)
    res[f"dw_{N}x{K}_hip_ms"] = timeit(lambda: torch.autograd.grad(y, (w, b), gy, retain_graph=True))
    res[f"dw_{N}x{K}_torch_ms"] = timeit(lambda: (gy.t() @ xi, gy.sum(0)))
    res[f"dw_{N}x{K}_hbm_floor_ms"] = 4.0 * rows * (N + K) / 8e12 * 1e3
for K, N in [(12, 36), (12, 48), (48, 12)]:
    xi = torch.randn(rows, K, device=dev)
    w = torch.randn(N, K, device=dev)
    b = torch.randn(N, device=dev)
    res[f"fwd_{K}x{N}_hip_ms"] = timeit(lambda: MF._tlin(xi, w, b, K, N))
    res[f"fwd_{K}x{N}_torch_ms"] = timeit(lambda: torch.nn.functional.linear(xi, w, b))
    res[f"fwd_{K}x{N}_hbm_floor_ms"] = 4.0 * rows * (N + K) / 8e12 * 1e3
xg = torch.randn(rows, 12, device=dev)
w1 = torch.randn(48, 12, device=dev)
b1 = torch.randn(48, device=dev)
res["fwd_gelu_12x48_hip_ms"] = timeit(lambda: MF._tlin(xg, w1, b1, 12, 48, epi=1))
res["fwd_gelu_12x48_torch_ms"] = timeit(lambda: torch.nn.functional.gelu(torch.nn.functional.linear(xg, w1, b1)))
fc1, fc2 = torch.nn.Linear(12, 48).to(dev), torch.nn.Linear(48, 12).to(dev)
act, drop = torch.nn.GELU(), torch.nn.Dropout(0.0)
xm = torch.randn(rows, 12, device=dev, requires_grad=True)
gm = torch.randn(rows, 12, device=dev)
res["mlp_fwdbwd_hip_ms"] = timeit(lambda: torch.autograd.backward(MF.mlp(xm, fc1, fc2, act, drop), gm))
res["mlp_fwdbwd_torch_ms"] = timeit(lambda: torch.autograd.backward(fc2(act(fc1(xm))), gm))
print(json.dumps({k: round(v, 4) for k, v in res.items()}))
