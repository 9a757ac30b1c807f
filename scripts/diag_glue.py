"""Shapes of the torch elementwise add / fill / copy ops in one C3 training step (diagnostic for the
glue kernels of the rocprof summaries).  usage: python scripts/diag_glue.py"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_neuroimage_amd import model as M  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
m = M.SwinFusion(**bench.model_kwargs(96)).to(dev)
A = torch.randn(4, 96, 96, 96, device=dev)
B = torch.randn(4, 96, 96, 96, device=dev)
y = torch.ones(4, 1, device=dev)
for _ in range(2):
    torch.nn.functional.binary_cross_entropy_with_logits(m(A, B)["binary_classification"], y).backward()
torch.cuda.synchronize()
for prm in m.parameters():
    prm.grad = None   # as the bench's zero_grad(set_to_none=True): no gradient-accumulation adds
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], record_shapes=True) as prof:
    torch.nn.functional.binary_cross_entropy_with_logits(m(A, B)["binary_classification"], y).backward()
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::copy_", "aten::zeros",
                   "aten::zeros_like", "aten::clone", "aten::contiguous", "aten::cat", "aten::mul", "aten::sum",
                   "aten::to", "aten::_to_copy", "aten::sub", "aten::div", "aten::index", "aten::where",
                   "aten::masked_fill", "aten::empty_strided", "aten::narrow_copy", "aten::slice_backward"):
        cnt[(ev.name, str(ev.input_shapes)[:120])] += 1
for (n, s), c in sorted(cnt.items(), key=lambda kv: -kv[1])[:60]:
    print(f"{c:5d}  {n:18s} {s}")
