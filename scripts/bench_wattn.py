"""Standalone timing of the window-attention kernels at the bench shape (B=4, 96^3, C=12, h=6,
window 6^3, shift 3), through the C ABI.  usage: python scripts/bench_wattn.py [reps]"""
import os
import sys
import json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
B, S, C, heads = 4, 96, 12, 6
geom = MF.WindowGeometry(B, (S, S, S), (6, 6, 6), (3, 3, 3))
rows = geom.tokens
torch.manual_seed(0)
qkv = torch.randn(rows, 3 * C, device=dev, requires_grad=True)
table = (torch.randn(geom.table_rows, heads, device=dev) * 0.02).requires_grad_(True)
g = torch.randn(rows, C, device=dev)
res = {}
for _ in range(2):
    out = MF.window_attention_self(qkv, table, geom, heads)
    out.backward(g)
torch.cuda.synchronize()
MF.KernelTimer.reset(); MF.KernelTimer.enabled = True
for _ in range(reps):
    out = MF.window_attention_self(qkv, table, geom, heads)
    out.backward(g)
MF.KernelTimer.enabled = False
summ = MF.KernelTimer.summary()
for k, v in summ.items():
    res[k] = dict(avg_ms=round(v["avg_ms"], 4), tflops=round(v["flops_per_launch"] / v["avg_ms"] / 1e9, 3))
print(json.dumps(dict(abl=os.environ.get("MMNI_WATTN_ABL", "0"), **res)))
