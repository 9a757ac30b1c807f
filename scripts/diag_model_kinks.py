"""Where do the fp32-vs-fp64 input-gradient differences of the 48^3 SwinFusion parity model sit?
(test_fullsize_gpu.py::test_swinfusion3d_full_depth_48).  Prints, per input, the max-norm and
L2 relative errors, how many voxels exceed 1e-4 of the max, and the bounding box of those voxels.
usage: python scripts/diag_model_kinks.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from multimodal_neuroimage_amd import model as M  # noqa: E402
from oracle import model as OM  # noqa: E402
from golden import recipe  # noqa: E402

dev = torch.device("cuda:0")
kw = dict(fine_tune_task="binary_classification", size_of_model="large", swin_embed_dim=12, drop_rate=0.0,
          attn_drop_rate=0.0, mlp_ratio=4.0, drop_path_rate=0.0, intermediate_vec=48, patch_size=4,
          window_size=6, no_init_weights=True, volume_size=48)
m = M.SwinFusion(**kw)
A = torch.from_numpy(recipe.randn(8100, (2, 48, 48, 48)))
Bv = torch.from_numpy(recipe.randn(8101, (2, 48, 48, 48)))
cfg = dict(window_size=6, Ex_depths=[6, 6], Fusion_depths=[2, 2, 2], Re_depths=[6, 6], heads=6,
           resolution=(12, 12, 12), head_patch=4)
tgt = torch.tensor([[1.0], [0.0]])
recipe.fill_params(m)
for mod in m.modules():
    if hasattr(mod, "drop_prob"):
        mod.drop_prob = 0.0
p = OM.params_of(m, torch.float64, dev)
ins64 = [t.to(dev).double().requires_grad_(True) for t in (A, Bv)]
OM.ATTN_CHUNK = 256
ref = OM.swinfusion_logits(p, *ins64, cfg)
torch.nn.functional.binary_cross_entropy_with_logits(ref, tgt.to(dev).double()).backward()
m = m.to(dev)
ins = [t.to(dev).requires_grad_(True) for t in (A, Bv)]
out = m(*ins)["binary_classification"]
torch.nn.functional.binary_cross_entropy_with_logits(out, tgt.to(dev)).backward()
torch.cuda.synchronize()
for name, a, r in zip("AB", ins, ins64):
    a, r = a.grad.double(), r.grad.double()
    d = (a - r).abs()
    mx = float(r.abs().max())
    big = (d > 1e-4 * mx).nonzero()
    print(f"input {name}: max-rel {float(d.max()) / mx:.3e}  L2-rel {float(d.norm() / r.norm()):.3e}  "
          f"voxels > 1e-4 max: {big.shape[0]}  of {d.numel()}")
    if big.shape[0]:
        print("   bbox lo", big.min(0).values.tolist(), "hi", big.max(0).values.tolist())
        flat = int(d.flatten().argmax())
        idx = []
        for s in reversed(d.shape):
            idx.append(flat % s)
            flat //= s
        print("   argmax", list(reversed(idx)))
