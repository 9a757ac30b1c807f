"""Oracle float ops vs fixtures generated from the reference (CPU, fp32, tolerance 1e-5 relative
to the output scale).  This pins the oracle; the GPU tests then check the HIP kernels against it."""
import json

import numpy as np
import pytest
import torch

import recipe
from _cases import wattn_meta, wattn_module, wattn_inputs, oracle_wattn_tokens
from oracle import ops as O
from multimodal_neuroimage_amd.modules import multihead_attention as MHA
from multimodal_neuroimage_amd.modules import position_embedding as PE

torch.set_num_threads(8)


def close(a, b, tol=1e-5):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-6)
    err = np.abs(a - b).max() / scale
    assert err <= tol, f"max rel err {err:.3e} > {tol:.1e}"


@pytest.mark.parametrize("name", ["f12s0", "f12s3", "f84s3", "c12s3", "c84s3", "v12s0", "v12s3", "v6s0", "v3s0"])
def test_oracle_window_attention_fwd_bwd(golden, name):
    case = wattn_meta(golden)[name]
    g = golden("wattn.npz")
    m = wattn_module(case)
    x, y, gout = wattn_inputs(golden, name, case)
    x.requires_grad_(True)
    if y is not None:
        y.requires_grad_(True)
    out = oracle_wattn_tokens(m, case, x, y)
    close(out.detach().numpy(), g[name + ".out"])
    (out * gout).sum().backward()
    close(x.grad.numpy(), g[name + ".dx"])
    if y is not None:
        close(y.grad.numpy(), g[name + ".dy"])
    for k, p in m.named_parameters():
        close(p.grad.numpy(), g[f"{name}.d.{k}"], tol=2e-5)


@pytest.mark.parametrize("T", [16, 368])
def test_oracle_mha(golden, T):
    g = golden("mha.npz")
    meta = json.loads(str(g["meta"]))[f"mha{T}"]
    mod = MHA.MultiheadAttention(84, 12)
    recipe.fill_params(mod)
    seed = meta["seed"]
    q, k, v = [torch.from_numpy(recipe.randn(seed + i, (T, 2, 84))).requires_grad_(True) for i in range(3)]
    E = 84
    W, b = mod.in_proj_weight, mod.in_proj_bias
    qp = torch.nn.functional.linear(q, W[:E], b[:E])
    kp = torch.nn.functional.linear(k, W[E:2 * E], b[E:2 * E])
    vp = torch.nn.functional.linear(v, W[2 * E:], b[2 * E:])
    o, w = O.mha_core(qp, kp, vp, 12, O.causal_diag(T, T))
    out = mod.out_proj(o)
    close(out.detach().numpy(), g[f"mha{T}.out"])
    wref = g[f"mha{T}.w"]
    close(w.detach().numpy()[:, :wref.shape[1], :wref.shape[2]], wref)
    gout = torch.from_numpy(recipe.randn(seed + 3, tuple(out.shape)))
    gw = torch.from_numpy(recipe.randn(seed + 4, tuple(w.shape)))
    ((out * gout).sum() + (w * gw).sum()).backward()
    for nm, t in (("dq", q), ("dk", k), ("dv", v)):
        close(t.grad.numpy(), g[f"mha{T}.{nm}"])


def test_oracle_positions(golden):
    g = golden("mha.npz")
    tok = torch.from_numpy(g["pe.tok"])
    pos = O.sinusoidal_positions(tok)
    tab = O.sinusoidal_table(int(pos.max()) + 1, 84)
    close(tab[pos.reshape(-1)].view(2, 30, 84).numpy(), g["pe.out"], tol=1e-6)


def test_product_positions_match_reference_on_cpu(golden):
    """The product SinusoidalPositionalEmbedding is plain torch (no HIP kernel); check it on CPU."""
    g = golden("mha.npz")
    pe = PE.SinusoidalPositionalEmbedding(84)
    close(pe(torch.from_numpy(g["pe.tok"])).numpy(), g["pe.out"], tol=1e-6)


def test_oracle_conv3d_matches_torch_conv2d_at_depth_one():
    """The channels-last conv oracle at D = 1, kd = 1 equals nn.Conv2d (the reference's 2D convs)."""
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(6, 12, 3, 1, 1)
    x = torch.randn(2, 6, 20, 24)
    ref = torch.nn.functional.leaky_relu(conv(x), 0.2)
    x_cl = x.permute(0, 2, 3, 1).unsqueeze(1)
    got = O.conv3d_cl(x_cl, conv.weight.unsqueeze(2), conv.bias, (1, 1, 1), (0, 1, 1), 0.2)
    close(got.squeeze(1).permute(0, 3, 1, 2).detach().numpy(), ref.detach().numpy(), tol=1e-6)


@pytest.mark.parametrize("kind,spatial,window,shift,chunk", [
    (0, (12, 12, 18), (6, 6, 6), (3, 3, 3), 5),
    (1, (6, 12, 12), (3, 6, 6), (1, 3, 3), 3),
    (0, (1, 12, 18), (1, 6, 6), (0, 3, 3), 4),
])
def test_chunked_oracle_equals_unchunked(kind, spatial, window, shift, chunk):
    """The checkpointed window-chunked oracle (used at full 96^3 size on the GPU) returns the same
    output and gradients as the one-shot restatement pinned by the fixtures above."""
    B, C, heads = 2, 12, 3
    g = torch.Generator().manual_seed(11)
    T = B * int(np.prod(spatial))
    Tsz = int(np.prod([2 * w - 1 for w in window]))
    base = [torch.randn(T, C, generator=g, dtype=torch.float64) for _ in range(3)]
    base.append(torch.randn(Tsz, heads, generator=g, dtype=torch.float64))
    tau0 = torch.rand(heads, generator=g, dtype=torch.float64) * 10 + 1
    gout = torch.randn(T, C, generator=g, dtype=torch.float64)
    res = []
    for ch in (None, chunk):
        leaves = [t.clone().requires_grad_(True) for t in base]
        tau = tau0.clone().requires_grad_(True) if kind == 1 else None
        out = O.window_attention(*leaves, B, spatial, window, shift, heads, kind, tau=tau, chunk=ch)
        (out * gout).sum().backward()
        res.append([out.detach()] + [t.grad for t in leaves] + ([tau.grad] if tau is not None else []))
    for a, b in zip(*res):
        torch.testing.assert_close(a, b, rtol=1e-12, atol=1e-12)
