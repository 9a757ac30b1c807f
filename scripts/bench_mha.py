"""Standalone timing of the crossmodal MHA kernels (through the C ABI) at the C4 / C5 shapes of
SURVEY §8d: E = 84 / 168, 12 heads, causal (diag 1 + |Tk - Tq|), T = 1728 (12^3 tokens) and
4096 (16^3), batch 4 per GPU.  usage: python scripts/bench_mha.py [reps] [T:E:dtype,...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
res = {}
only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else None
for T, E, dt in [(1728, 84, torch.float32), (1728, 168, torch.float32), (4096, 84, torch.float32),
                 (4096, 84, torch.bfloat16), (4096, 168, torch.bfloat16), (1728, 84, torch.bfloat16)]:
    if only is not None and f"{T}:{E}:{str(dt).split('.')[-1]}" not in only:
        continue
    B, heads = 4, 12
    g = torch.Generator(device=dev).manual_seed(T + E)
    q, k, v = [torch.randn(T, B, E, device=dev, generator=g).to(dt).requires_grad_(True) for _ in range(3)]
    go = torch.randn(T, B, E, device=dev, generator=g).to(dt)
    diag = 1
    for _ in range(2):
        out, lse = MF.mha_core(q, k, v, heads, diag)
        out.backward(go)
    torch.cuda.synchronize()
    MF.KernelTimer.reset()
    MF.KernelTimer.enabled = True
    for _ in range(reps):
        out, lse = MF.mha_core(q, k, v, heads, diag)
        out.backward(go)
    MF.KernelTimer.enabled = False
    for name, s in MF.KernelTimer.summary().items():
        # causal: about half of the 4*T^2*E (fwd) / 10*T^2*E (bwd) algorithmic FLOPs are useful
        res[f"T{T}_E{E}_{name}"] = dict(avg_ms=round(s["avg_ms"], 4),
                                        tflops_full=round(s["flops_per_launch"] / s["avg_ms"] / 1e9, 2),
                                        tflops_causal=round(0.5 * s["flops_per_launch"] / s["avg_ms"] / 1e9, 2))
print(json.dumps(res))
