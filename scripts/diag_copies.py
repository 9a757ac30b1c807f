"""Which torch ops launch the device-to-device copies (rocprof `__amd_rocclr_copyBuffer`) and the
fills of one C3 training step?  usage: python scripts/diag_copies.py"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import model as M  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
m = M.SwinFusion(**bench.model_kwargs(96)).to(dev)
opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-5)
A = torch.randn(4, 96, 96, 96, device=dev)
B = torch.randn(4, 96, 96, 96, device=dev)
y = torch.ones(4, 1, device=dev)
lossf = torch.nn.BCEWithLogitsLoss()


def step():
    opt.zero_grad(set_to_none=True)
    lossf(m(A, B)["binary_classification"], y).backward()
    opt.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    for k in getattr(ev, "kernels", []) or []:
        n = k.name
        if "Memcpy" in n or "copyBuffer" in n or "Fill" in n or "fill" in n:
            cnt[(ev.name, str(ev.input_shapes)[:90], n[:40])] += 1
for (op, shp, kn), c in sorted(cnt.items(), key=lambda kv: -kv[1])[:40]:
    print(f"{c:5d}  {op:28s} {kn:40s} {shp}")
dev_cnt = collections.Counter(e.name[:60] for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA)
print("--- device events")
for n, c in dev_cnt.most_common(25):
    print(f"{c:5d}  {n}")
