"""Standalone timing of the fused LayerNorm + MLP + residual kernels (mlp.hip, LN variants) at the
C3 row count (4 x 96^3 tokens, C = 12, hidden 48), with the library MMNI_LIB selects.
usage: python scripts/bench_lnmlp.py [reps]"""
import json
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
rows, C, H = 4 * 96 ** 3, 12, 48
torch.manual_seed(0)
norm = torch.nn.LayerNorm(C).to(dev)
mod = types.SimpleNamespace(fc1=torch.nn.Linear(C, H).to(dev), fc2=torch.nn.Linear(H, C).to(dev),
                            act=torch.nn.GELU(), drop=torch.nn.Dropout(0.0))
x = torch.randn(rows, C, device=dev, requires_grad=True)
g = torch.randn(rows, C, device=dev)
assert MF.ln_mlp_ok(x, norm, mod)
for _ in range(2):
    MF.ln_mlp(x, norm, mod).backward(g)
torch.cuda.synchronize()
MF.KernelTimer.reset()
MF.KernelTimer.enabled = True
for _ in range(reps):
    MF.ln_mlp(x, norm, mod).backward(g)
MF.KernelTimer.enabled = False
out = {"lib": os.environ.get("MMNI_LIB", "default")}
for k, v in MF.KernelTimer.summary().items():
    out[k] = round(v["avg_ms"] * 1e3, 1)
print(json.dumps(out))
