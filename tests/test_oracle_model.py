"""Pins the functional oracle models (oracle/model.py) to the REFERENCE's own outputs
(tests/golden/models.npz, made by tests/golden/make_golden.py from the reference's model.py):
same recipe parameters and inputs, oracle in float64 on the CPU.

Logits / input grads must agree to fp32 round-off.  Parameter grads: the golden file is the
reference's fp32 result, whose own error on cancellation-heavy grads (deep Swin-V2 logit_scale /
q_bias) reaches ~2.4e-3 of the tensor max, so the elementwise bar there is 5e-3."""
import json

import numpy as np
import pytest
import torch

import recipe
from multimodal_neuroimage_amd import model as M
from oracle import model as OM

SF_CFG = dict(window_size=6, Ex_depths=[6, 6], Fusion_depths=[2, 2, 2], Re_depths=[6, 6], heads=6,
              resolution=(12, 12), head_patch=7)


def rel(a, b):
    a = torch.as_tensor(np.asarray(a, np.float64))
    b = torch.as_tensor(np.asarray(b, np.float64))
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _run(golden, name):
    g = golden("models.npz")
    kw = json.loads(str(g["meta"]))[name]["kwargs"]
    if name == "swinfusion":
        m = M.SwinFusion(**kw)
        recipe.fill_params(m)
        A = torch.from_numpy(recipe.randn(4000, (2, 84, 84))).double().requires_grad_(True)
        Bv = torch.from_numpy(recipe.randn(4001, (2, 84, 84))).double().requires_grad_(True)
        p = OM.params_of(m)
        out = OM.swinfusion_logits(p, A, Bv, SF_CFG)
        tgt = torch.tensor([[1.0], [0.0]], dtype=torch.float64)
        inputs = {"dA": A, "dB": Bv}
    else:
        m = M.SwinTransformerV2(**kw)
        recipe.fill_params(m)
        X = torch.from_numpy(recipe.randn(4100, (4, 84, 84))).double().requires_grad_(True)
        p = OM.params_of(m)
        out = OM.swin_v2_logits(p, "", X, kw["patch_size"], kw["window_size"])
        tgt = torch.tensor([[1.0], [0.0], [1.0], [0.0]], dtype=torch.float64)
        inputs = {"dX": X}
    torch.nn.functional.binary_cross_entropy_with_logits(out, tgt).backward()
    return g, out, inputs, p


@pytest.mark.parametrize("name", ["swinfusion", "swinv2"])
def test_oracle_model_matches_reference(golden, name):
    g, out, inputs, p = _run(golden, name)
    assert rel(out.detach(), g[f"{name}.logits"]) < 1e-5
    for k, t in inputs.items():
        assert rel(t.grad, g[f"{name}.{k}"]) < 1e-4, k
    names = list(g[f"{name}.gnames"])
    gsq = g[f"{name}.gsq"]
    for i, n in enumerate(names):
        grad = p[n].grad if p[n].grad is not None else torch.zeros_like(p[n])
        key = f"{name}.d.{n}"
        if key in g.files:
            assert rel(grad, g[key]) < 5e-3, n
        else:
            nrm = float(grad.pow(2).sum().sqrt())
            assert abs(nrm - np.sqrt(gsq[i])) <= 1e-3 * max(np.sqrt(gsq[i]), 1e-12) + 1e-12, n


def test_oracle_crossmodal_head_matches_reference(golden):
    """The oracle's crossmodal encoder stack (used for the C4 composite) against the reference's
    Transformer_Net_Cross_Attention logits and embedding (default options: proj_l Conv1d,
    12 layers, 12 heads, causal)."""
    g = golden("models.npz")
    kw = json.loads(str(g["meta"]))["crossmodal"]["kwargs"]
    m = M.Transformer_Net_Cross_Attention(**kw)
    recipe.fill_params(m)
    p = OM.params_of(m)
    xl = torch.from_numpy(recipe.randn(4200, (2, 368, 84))).double()
    xu = torch.from_numpy(recipe.randn(4201, (2, 368, 84))).double()
    with torch.no_grad():
        emb, out = OM.crossmodal_head(p, "", xl, xu, kw["nlevels"], kw["num_heads_mult"], kw["feature_map_gen"],
                                      kw["attn_mask"])
    assert rel(out, g["crossmodal.logits"]) < 1e-5
    assert rel(emb, g["crossmodal.emb"]) < 1e-5
