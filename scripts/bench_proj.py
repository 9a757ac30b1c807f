"""Timing of the block's attn.proj (12 -> 12 token Linear + residual, tokenlinear.hip) forward and
backward at the C3 row count, with the library MMNI_LIB selects.  usage: python scripts/bench_proj.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
rows, C = 4 * 96 ** 3, 12
torch.manual_seed(0)
lin = torch.nn.Linear(C, C).to(dev)
x = torch.randn(rows, C, device=dev, requires_grad=True)
r = torch.randn(rows, C, device=dev, requires_grad=True)
g = torch.randn(rows, C, device=dev)
for _ in range(2):
    MF.linear(x, lin, residual=r).backward(g)
torch.cuda.synchronize()
MF.KernelTimer.reset()
MF.KernelTimer.enabled = True
for _ in range(reps):
    MF.linear(x, lin, residual=r).backward(g)
MF.KernelTimer.enabled = False
out = {"lib": os.environ.get("MMNI_LIB", "default")}
for k, v in MF.KernelTimer.summary().items():
    out[k] = round(v["avg_ms"] * 1e3, 1)
print(json.dumps(out))
