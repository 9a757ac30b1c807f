"""Timing of the token MLP at the C3 shape (4 x 96^3 tokens, C = 12, hidden 48): the one-kernel
MFMA path (mlp.hip) vs the token-linear path, forward + backward.  usage: python scripts/bench_mlp.py"""
import json
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import functional as MF

dev = torch.device("cuda:0")
rows, C, H = 4 * 96 ** 3, 12, 48
torch.manual_seed(0)
fc1, fc2 = torch.nn.Linear(C, H).to(dev), torch.nn.Linear(H, C).to(dev)
x = torch.randn(rows, C, device=dev, requires_grad=True)
r = torch.randn(rows, C, device=dev, requires_grad=True)
g = torch.randn(rows, C, device=dev)
res = {}
for name, fn in (("mfma", lambda: MF.mlp(x, fc1, fc2, torch.nn.GELU(), torch.nn.Dropout(0.0), residual=r)),
                 ("tokenlinear", lambda: MF._Mlp.apply(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, r))):
    for _ in range(2):
        fn().backward(g)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    MF.KernelTimer.reset(); MF.KernelTimer.enabled = True
    t0.record()
    for _ in range(5):
        fn().backward(g)
    t1.record()
    MF.KernelTimer.enabled = False
    summ = MF.KernelTimer.summary()
    res[name] = dict(ms_fwd_bwd=round(t0.elapsed_time(t1) / 5, 3),
                     kernels={k: round(v["avg_ms"], 4) for k, v in summ.items()})
print(json.dumps(res))
