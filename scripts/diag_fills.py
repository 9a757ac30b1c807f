"""Count the torch fill / add launches of one SwinFusion-3D training step by Python call site
(diagnostic for the FillFunctor / CUDAFunctor_add kernels in the rocprof summaries)."""
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import model as M  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
m = M.SwinFusion(**bench.model_kwargs(96)).to(dev)
A = torch.randn(1, 96, 96, 96, device=dev)
B = torch.randn(1, 96, 96, 96, device=dev)
y = torch.ones(1, 1, device=dev)
for _ in range(2):
    torch.nn.functional.binary_cross_entropy_with_logits(m(A, B)["binary_classification"], y).backward()
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                            with_stack=True) as prof:
    torch.nn.functional.binary_cross_entropy_with_logits(m(A, B)["binary_classification"], y).backward()
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::add", "aten::add_"):
        st = [s for s in (ev.stack or []) if "multimodal_neuroimage_amd" in s or "bench" in s]
        cnt[(ev.name, st[0] if st else "(autograd engine / no python frame)")] += 1
for (n, site), c in cnt.most_common(30):
    print(f"{c:5d}  {n:16s} {site}")
