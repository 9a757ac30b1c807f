"""One C3 training step under torch.profiler: the framework-level (aten) ops around the HIP kernels,
grouped by input shape with the Python source line, to find elementwise adds / fills that the
fused kernels could absorb.  usage: python scripts/torch_prof_step.py [out.txt]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multimodal_neuroimage_amd import model as M  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/torch_prof.txt"
dev = torch.device("cuda:0")
m = M.SwinFusion(**bench.model_kwargs(96)).to(dev)
for mod in m.modules():
    if hasattr(mod, "drop_prob"):
        mod.drop_prob = 0.0
opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
A, B, y = bench.synthetic_pairs(4, 96, dev, 0)
lossf = torch.nn.functional.binary_cross_entropy_with_logits


def step():
    opt.zero_grad(set_to_none=True)
    loss = lossf(m(A, B)["binary_classification"], y)
    loss.backward()
    opt.step()


step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
with open(out, "w") as f:
    f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="count", row_limit=60))
    f.write("\n\n")
    f.write(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=40))
print("wrote", out)
