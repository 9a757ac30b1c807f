"""One training step under torch.profiler: the framework-level (aten) ops around the HIP kernels,
grouped by input shape and by Python stack, with their device time, to find the casts, reductions,
adds and fills that the fused kernels could absorb.
usage: python scripts/torch_prof_step.py [out.txt] [c3|c4|c5]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multimodal_neuroimage_amd import model as M  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/torch_prof.txt"
cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
dev = torch.device("cuda:0")
if cfg in ("c4", "c5"):
    size = 128 if cfg == "c5" else 96
    m = M.SwinCrossmodal3D(**(bench.c5_kwargs if cfg == "c5" else bench.c4_kwargs)(size)).to(dev)
    A, B, y = bench.synthetic_pairs(8 if cfg == "c5" else 4, size, dev, 0,
                                    size_b=size * 3 // 4 if cfg == "c5" else None)
else:
    m = M.SwinFusion(**bench.model_kwargs(96)).to(dev)
    A, B, y = bench.synthetic_pairs(4, 96, dev, 0)
for mod in m.modules():
    if hasattr(mod, "drop_prob"):
        mod.drop_prob = 0.0
opt = torch.optim.AdamW(m.parameters(), lr=1e-4, fused=True)
lossf = torch.nn.functional.binary_cross_entropy_with_logits


def step():
    opt.zero_grad(set_to_none=True)
    loss = lossf(m(A, B)["binary_classification"], y)
    loss.backward()
    opt.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
with open(out, "w") as f:
    f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total", row_limit=80))
    f.write("\n\n")
    f.write(prof.key_averages(group_by_stack_n=5).table(sort_by="self_device_time_total", row_limit=60))
print("wrote", out)
