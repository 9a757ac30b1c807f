"""C5 bf16-head gradient error profile against the fp64 oracle (diagnostic; prints rel-L2 / max-rel
per parameter group).  usage: python scripts/diag_c5_grads.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import recipe  # noqa: E402
from multimodal_neuroimage_amd import model as M  # noqa: E402
from oracle import model as OM  # noqa: E402

dev = torch.device("cuda:0")
kw = dict(fine_tune_task="binary_classification", volume_size=64, patch_size=8, swin_embed_dim=12, window_size=4,
          swin_heads=3, cross_heads=6, swin_depth=2, mlp_ratio=4.0, intermediate_vec=84, num_heads_mult=12, nlevels=2,
          attn_dropout=0.0, attn_dropout_u=0.0, relu_dropout=0.0, res_dropout=0.0, embed_dropout=0.0, out_dropout=0.0,
          attn_mask=True, mixing="U2L_and_L2U", concat_method="concat", fmri_type="divided_frequency",
          volume_size_B=48, patch_size_B=6)
from multimodal_neuroimage_amd.modules import multihead_attention as MHA_MOD  # noqa: E402
_kernel_core = MHA_MOD.mha_core


def torch_core(q, k, v, heads, diag, scale, dropout=0.0, seed=0):
    """the reference's bmm -> fp32 softmax -> type_as -> bmm (multihead_attention.py:109-125) in torch"""
    Tq, B, E = q.shape
    Tk = k.shape[0]
    d = E // heads
    qh = (q * scale).reshape(Tq, B * heads, d).transpose(0, 1)
    kh = k.reshape(Tk, B * heads, d).transpose(0, 1)
    vh = v.reshape(Tk, B * heads, d).transpose(0, 1)
    w = torch.bmm(qh, kh.transpose(1, 2))
    if diag > 0:
        w = w + torch.triu(torch.full((Tq, Tk), float("-inf"), device=q.device), diag).to(w.dtype)
    w = torch.softmax(w.float(), dim=-1).type_as(w)
    o = torch.bmm(w, vh).transpose(0, 1).reshape(Tq, B, E)
    lse = torch.zeros(B, heads, Tq, device=q.device)
    return o, lse


res = {}
for hd in ("fp32", "bf16", "bf16-torch-attn"):
    MHA_MOD.mha_core = torch_core if hd == "bf16-torch-attn" else _kernel_core
    m = M.SwinCrossmodal3D(head_dtype=hd[:4], **kw)
    recipe.fill_params(m)
    A = torch.from_numpy(recipe.randn(5100, (2, 64, 64, 64)))
    Bv = torch.from_numpy(recipe.randn(5101, (2, 48, 48, 48)))
    tgt = torch.tensor([[1.0], [0.0]])
    if hd == "fp32":
        p = OM.params_of(m)
        cfg = dict(patch=8, patch_B=6, window_size=4, swin_heads=3, cross_heads=6, depth=2, layers=2, heads=12)
        ref = OM.swin_crossmodal_logits(p, A.double(), Bv.double(), cfg)
        torch.nn.functional.binary_cross_entropy_with_logits(ref, tgt.double()).backward()
    m = m.to(dev)
    out = m(A.to(dev), Bv.to(dev))["binary_classification"]
    torch.nn.functional.binary_cross_entropy_with_logits(out, tgt.to(dev)).backward()
    torch.cuda.synchronize()
    for k, prm in m.named_parameters():
        if prm.grad is None or p[k].grad is None:
            continue
        a, b = prm.grad.double().cpu(), p[k].grad
        l2 = float((a - b).norm() / max(float(b.norm()), 1e-30))
        mx = float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))
        res.setdefault(k, {})[hd] = (l2, mx)
worst = sorted(res.items(), key=lambda kv: -kv[1]["bf16"][0])[:25]
for k, v in worst:
    t = v["bf16-torch-attn"]
    print(f"{k:62s} fp32 {v['fp32'][0]:.1e} | bf16 kernels l2 {v['bf16'][0]:.2e} max {v['bf16'][1]:.2e} | "
          f"bf16 torch-attn l2 {t[0]:.2e} max {t[1]:.2e}")
import numpy as np  # noqa: E402
for mode in ("bf16", "bf16-torch-attn"):
    l2s = np.array([v[mode][0] for v in res.values()])
    print(mode, "median l2", float(np.median(l2s)), "p90", float(np.percentile(l2s, 90)), "max", float(l2s.max()))
