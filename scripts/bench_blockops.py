"""Standalone timing of the fused LN + Linear kernels (blockops.hip) at the C3 row count
(4 x 96^3 tokens), through the C ABI, with the library MMNI_LIB selects.
usage: python scripts/bench_blockops.py [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
rows = 4 * 96 ** 3
torch.manual_seed(0)
x = torch.randn(rows, 12, device=dev, requires_grad=True)
norm = torch.nn.LayerNorm(12).to(dev)
MF.KernelTimer.reset()
for N in (12, 24, 36):
    lin = torch.nn.Linear(12, N).to(dev)
    g = torch.randn(rows, N, device=dev)
    gr = torch.randn(rows, 12, device=dev)

    def step():
        # as in the blocks: the residual view's gradient (dres) joins inside the backward
        y, xr = MF.ln_linear(x, norm, lin, passthrough=True)
        torch.autograd.backward([y, xr], [g, gr])
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    MF.KernelTimer.enabled = True
    for _ in range(reps):
        step()
    MF.KernelTimer.enabled = False
out = {"lib": os.environ.get("MMNI_LIB", "default")}
for k, v in MF.KernelTimer.summary().items():
    out[k] = round(v["avg_ms"] * 1e3, 1)
print(json.dumps(out))
