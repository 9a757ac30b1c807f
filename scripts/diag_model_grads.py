"""Diagnostic: SwinFusion golden case — product (GPU, if present) and reference-fp32 golden
grads, each against the fp64 oracle.  Prints the worst parameters."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import recipe  # noqa: E402
from multimodal_neuroimage_amd import model as M  # noqa: E402
from oracle import model as OM  # noqa: E402

g = np.load(os.path.join(ROOT, "tests/golden/models.npz"))
kw = json.loads(str(g["meta"]))["swinfusion"]["kwargs"]
m = M.SwinFusion(**kw).eval()
recipe.fill_params(m)
A = torch.from_numpy(recipe.randn(4000, (2, 84, 84)))
Bv = torch.from_numpy(recipe.randn(4001, (2, 84, 84)))
tgt = torch.tensor([[1.0], [0.0]])
p = OM.params_of(m, torch.float64)
cfg = dict(window_size=6, Ex_depths=[6, 6], Fusion_depths=[2, 2, 2], Re_depths=[6, 6], heads=6,
           resolution=(12, 12), head_patch=7)
out64 = OM.swinfusion_logits(p, A.double(), Bv.double(), cfg)
torch.nn.functional.binary_cross_entropy_with_logits(out64, tgt.double()).backward()
print("oracle64 vs golden logits", float((out64.detach() - torch.from_numpy(g["swinfusion.logits"])).abs().max()))
ours = None
if torch.cuda.is_available():
    md = m.cuda()
    out = md(A.cuda(), Bv.cuda())["binary_classification"]
    torch.nn.functional.binary_cross_entropy_with_logits(out, tgt.cuda()).backward()
    ours = {k: v.grad.detach().double().cpu() for k, v in md.named_parameters() if v.grad is not None}


def rel(a, b):
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


rows = []
for n, t in p.items():
    key = "swinfusion.d." + n
    if t.grad is None:
        continue
    ge = rel(torch.from_numpy(g[key]).double(), t.grad) if key in g.files else float("nan")
    oe = rel(ours[n], t.grad) if ours is not None and n in ours else float("nan")
    rows.append((oe if ours is not None else ge, ge, oe, n))
rows.sort(reverse=True)
for r in rows:
    if "layers.2.blocks.3.attn.logit_scale" in r[3] or "layers.2.blocks.4.attn.logit_scale" in r[3]:
        print("SPECIFIC", r)
print(f"{'ours_vs_fp64':>14} {'golden_vs_fp64':>15}  param")
for _, ge, oe, n in rows[:25]:
    print(f"{oe:14.3e} {ge:15.3e}  {n}")
